#!/usr/bin/env python3
"""Where one C2 query's time goes (r06): the whole ve.query, the AQL chain alone (run_direct: ctypes
call + GPU + the spin wait), and the Python part alone (run_direct replaced by a no-op), medians over
N queries of the bench's 20 reference rows; plus each step of the chain alone.

    python3 tools/c2_split.py [N]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n=2000):
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    with open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")) as f:
        g = json.load(f)
    m = get_example_model("munin")
    q = g["variables"]
    rows = [r["evidence"] for r in g["rows"]]
    ve = VariableElimination(m)
    for k in range(100):
        ve.query(q, rows[k % 20], show_progress=False)
    torch.cuda.synchronize()
    runner, = ve._compiled.values()
    prog = runner.plan.__dict__["_q1"]["joint"][0]

    def timeit(fn, reps):
        ts = []
        for k in range(reps):
            t0 = time.perf_counter()
            fn(k)
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e6

    out = {"whole_us": timeit(lambda k: ve.query(q, rows[k % 20], show_progress=False), n),
           "chain_us": timeit(lambda k: prog.run_direct(), n)}
    real = prog.run_direct
    prog.run_direct = lambda: None
    try:
        out["python_us"] = timeit(lambda k: ve.query(q, rows[k % 20], show_progress=False), n)
    finally:
        prog.run_direct = real
    out["launches"] = len(prog._direct)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
