#!/usr/bin/env python3
"""munin belief propagation on the device: min-fill junction tree (1,033 cliques, max 2.74 M states),
one calibration with the C2 evidence (100 leaf findings), the C2 root's marginal compared with the
reference's VE posterior (tests/golden/munin_c2_query.json).  Prints one JSON line.
    python tools/munin_bp.py [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import BeliefPropagation
    from pgmpy_amd.utils import get_example_model

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_query.json")))
    m = get_example_model("munin")
    t0 = time.perf_counter()
    bp = BeliefPropagation(m)
    t1 = time.perf_counter()
    r = bp.query(g["variables"], g["evidence"], show_progress=False)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        r = bp.query(g["variables"], g["evidence"], show_progress=False)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    got = np.asarray(r.values, dtype=float).ravel()
    want = np.asarray(g["result"]["values"], dtype=float).ravel()
    print(json.dumps({"jt_build_s": t1 - t0, "first_query_s": t2 - t1, "query_s": float(np.median(ts)),
                      "cliques": len(bp.junction_tree.nodes()) if hasattr(bp, "junction_tree") else None,
                      "max_abs_err": float(np.abs(got - want).max()), "got": got.tolist(), "want": want.tolist()}))


if __name__ == "__main__":
    main()
