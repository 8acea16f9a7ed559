#!/usr/bin/env python3
"""cProfile of the C2 query loop (munin, the reference's 20 rows, compiled plan cached): host time split."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import gc

    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")))
    q = g["variables"]
    rows = [r["evidence"] for r in g["rows"]]
    ve = VariableElimination(get_example_model("munin"))
    for r in rows:
        ve.query(q, r, show_progress=False)
    torch.cuda.synchronize()
    gc.collect()
    t0 = time.perf_counter()
    for k in range(1000):
        ve.query(q, rows[k % 20], show_progress=False)
    print("plain us/query", (time.perf_counter() - t0) / 1000 * 1e6)
    pr = cProfile.Profile()
    pr.enable()
    for k in range(1000):
        ve.query(q, rows[k % 20], show_progress=False)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    print(s.getvalue())


if __name__ == "__main__":
    main()
