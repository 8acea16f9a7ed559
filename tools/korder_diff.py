import json, os, sys
import numpy as np
sys.path.insert(0, "/root/repo") if os.path.isdir("/root/repo") else None
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
import torch
from pgmpy_amd.inference import VariableElimination
from pgmpy_amd.utils import get_example_model
g = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")))
ve = VariableElimination(get_example_model("munin"))
r = ve.query(g["variables"], g["rows"][0]["evidence"], show_progress=False)
torch.cuda.synchronize()
runner, = ve._compiled.values()
prog = runner.plan.__dict__["_q1"]["joint"][0]
prog.run_direct()
torch.cuda.synchronize()
ts = [t for t in prog._keep if isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64]
np.savez(sys.argv[1], *[t.detach().cpu().numpy().ravel() for t in ts])
print(len(ts), "tensors", np.asarray(r.values).ravel()[:4], prog.notes)
