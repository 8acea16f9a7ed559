#!/usr/bin/env python3
"""Config 4 as one calibration: pathfinder BeliefPropagation(min-fill JT).calibrate() through the
API (per-message DiscreteFactor ops on the device), and the compiled batched schedule at 1 row
(graph replay).  Prints one JSON line.  python tools/c4_single.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import pandas as pd
    import torch

    from pgmpy_amd.inference import BeliefPropagation
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("pathfinder")
    bp = BeliefPropagation(m)
    t0 = time.perf_counter()
    bp.calibrate()  # first: per-message path (auto mode)
    torch.cuda.synchronize()
    first_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    bp.calibrate()  # second: records + compiles the schedule
    torch.cuda.synchronize()
    second_s = time.perf_counter() - t0
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        bp.calibrate()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    api_s = float(np.median(ts))
    bjt = BatchedJunctionTree(bp.junction_tree)
    df = pd.DataFrame({"F1": [np.nan]}, dtype=object)
    cal = bjt.calibrate_frame(df)
    torch.cuda.synchronize()
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        cal = bjt.calibrate_frame(df)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"api_first_calibrate_s": first_s, "api_second_calibrate_s (compile)": second_s,
                      "api_calibrate_s": api_s, "schedule_1row_s": float(np.median(ts)),
                      "reference_calibrate_s": "1.66-1.96 (SURVEY 8(d))"}))


if __name__ == "__main__":
    main()
