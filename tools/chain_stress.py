#!/usr/bin/env python3
"""Stress of the single-query AQL chain: 50,000 munin C2 queries (20 packets each, the 256-signal ring
and the 4,096-slot queue wrap many times) and 100,000 alarm queries, every 997th result and the last ones
checked against the reference goldens."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from tests.goldens import fac_values, load_json

    g = load_json("munin_c2_rows.json")
    q = g["variables"]
    ve = VariableElimination(get_example_model("munin"))
    t0 = time.perf_counter()
    bad = 0
    for k in range(50_000):
        row = g["rows"][k % 20]
        r = ve.query(q, row["evidence"], show_progress=False)
        if k % 997 == 0 or k >= 49_980:
            bad += not np.allclose(np.asarray(r.values).ravel(), fac_values(row["root"]), rtol=1e-6, atol=1e-12)
    print(f"c2: 50000 queries in {time.perf_counter() - t0:.1f} s, mismatches {bad}", flush=True)
    a = load_json("alarm_queries.json")
    va = VariableElimination(get_example_model("alarm"))
    pats = a["patterns"]
    t0 = time.perf_counter()
    bad = 0
    for k in range(100_000):
        p = pats[k % len(pats)]
        sep = va.query(p["variables"], p["evidence"], joint=False, show_progress=False)
        if k % 997 == 0 or k >= 99_950:
            for v in p["variables"]:
                bad += not np.allclose(np.asarray(sep[v].values), fac_values(p["marginals"][v]), atol=1e-10, rtol=0)
    torch.cuda.synchronize()
    print(f"alarm: 100000 queries in {time.perf_counter() - t0:.1f} s, mismatches {bad}", flush=True)
    print("direct:", next(iter(ve._compiled.values())).plan.__dict__["_progs"].popitem()[1][0].direct_note)


if __name__ == "__main__":
    main()
