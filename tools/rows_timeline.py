#!/usr/bin/env python3
"""Per-wave timeline of the affine row kernel (C3 template, 100k rows) from s_memrealtime stamps.

    python -m pgmpy_amd.build --timeline        # lib/libpgmhip_timeline.so (-DPGM_ROWS_TIMELINE)
    PGM_LIB_PATH=pgmpy_amd/lib/libpgmhip_timeline.so python tools/rows_timeline.py [rows]

The timeline build of the kernel writes [entry, ready, stores issued, stores acked, HW_ID, XCC_ID]
per wave into the gap buffer; this prints the distribution (100 MHz ticks -> us) relative to the
earliest wave entry of the launch.
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    assert "timeline" in os.environ.get("PGM_LIB_PATH", ""), "run against the timeline build (see docstring)"
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, rows, seed=42)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    d = upload_codes(np.ascontiguousarray(codes[[pos[v] for v in obs]]))
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    out = plan.alloc_outputs(rows, marginals=True)
    L = N.lib()
    n_waves = ((rows + 63) // 64) * 3
    tl = torch.zeros(n_waves * 6 + 64, dtype=torch.float64, device="cuda")
    plan.run(d, rows, 0, rows, out)  # creates the plan's device handle
    for rep in range(6):
        N.check(L.pgm_rows_plan_run(plan._handle,
                                    N.ROWS_MARGINALS, N.ptr(d), rows, 0, rows, N.ptr(out["marg"]), None,
                                    rows, None, N.ptr(tl), None, N.stream_handle()), "rows_plan_run")
    torch.cuda.synchronize()
    t = tl[: n_waves * 6].view(n_waves, 6).cpu().numpy()
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # 100 MHz
    entry, ready, issued, done = us(t[:, 0]), us(t[:, 1]), us(t[:, 2]), us(t[:, 3])
    pct = lambda a: [round(float(np.percentile(a, q)), 2) for q in (0, 10, 50, 90, 100)]
    res = {
        "waves": int(len(t)), "span_us": round(float(done.max()), 2),
        "entry_pct_us": pct(entry), "ready_minus_entry_pct_us": pct(ready - entry),
        "issued_minus_ready_pct_us": pct(issued - ready), "acked_minus_issued_pct_us": pct(done - issued),
        "done_pct_us": pct(done),
        "xcc_ids": sorted({int(x) & 15 for x in t[:, 5]}),
    }
    # waves entering per 0.5 us bin (dispatch rate)
    h, _ = np.histogram(entry, bins=np.arange(0, entry.max() + 0.5, 0.5))
    res["entries_per_0.5us"] = h.tolist()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
