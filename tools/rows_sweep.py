#!/usr/bin/env python3
"""Sweep the fused row kernel over batch sizes / variants (HIP-event timing, same stream).

    python tools/rows_sweep.py [--rows 100000 1000000 4000000] [--reps 20]
Prints one JSON line per (rows, variant): kernel us, rows/s, GB/s (143 B/row algorithmic).
"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="*", default=[100_000, 1_000_000, 4_000_000])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch

    from bench import HipTimer
    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.batch import upload_codes
    from pgmpy_amd.inference.plan import PatternPlan
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    base_rows = 100_000
    codes, nodes = forward_sample_codes(m, base_rows, seed=42)
    obs = [v for v in nodes if v not in missing]
    pos = {v: i for i, v in enumerate(nodes)}
    ev = np.ascontiguousarray(codes[[pos[v] for v in obs]])
    plan = PatternPlan(m, missing, obs, {v: i for i, v in enumerate(obs)})
    for rows in a.rows:
        rep = -(-rows // base_rows)
        d = upload_codes(np.tile(ev, (1, rep))[:, :rows])
        for name, extra, outs in (("lds_values", 0, dict(marginals=True)),
                                  ("global_values", N.ROWS_VALUES_GLOBAL, dict(marginals=True)),
                                  ("map_only", 0, dict(marginals=False, map_=True))):
            plan.extra_mode = extra
            out = plan.alloc_outputs(rows, **outs)
            for _ in range(3):
                plan.run(d, rows, 0, rows, out)
            t = HipTimer()
            t.start()
            for _ in range(a.reps):
                plan.run(d, rows, 0, rows, out)
            us = t.stop_ms() * 1e3 / a.reps
            bpr = plan.algorithmic_bytes_per_row(marginals=outs.get("marginals", False), map_=outs.get("map_", False))
            print(json.dumps({"rows": rows, "variant": name, "kernel_us": us, "rows_per_s": rows / us * 1e6,
                              "GBps": bpr * rows / us / 1e3, "bytes_per_row": bpr}), flush=True)
        plan.extra_mode = 0
        del d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
