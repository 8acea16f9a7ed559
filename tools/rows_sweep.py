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
    ap.add_argument("--variants", nargs="*", default=None, help="subset of variant names (default: all)")
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
        # practical floor: torch's fill of the same marginal output (write-only, same bytes)
        if a.variants is None or "torch_fill_floor" in a.variants:
            mt = plan.alloc_outputs(rows, marginals=True)["marg"]
            for _ in range(3):
                mt.fill_(0.5)
            t = HipTimer()
            t.start()
            for _ in range(a.reps):
                mt.fill_(0.5)
            us = t.stop_ms() * 1e3 / a.reps
            print(json.dumps({"rows": rows, "variant": "torch_fill_floor", "kernel_us": us,
                              "GBps": mt.numel() * 8 / us / 1e3}), flush=True)
            del mt
        for name, extra, outs in (("lds_values", 0, dict(marginals=True)),
                                  ("lds_one_group", N.ROWS_ONE_GROUP, dict(marginals=True)),
                                  ("generic_kernel", N.ROWS_GENERIC, dict(marginals=True)),
                                  ("global_values", N.ROWS_VALUES_GLOBAL, dict(marginals=True)),
                                  ("map_only", 0, dict(marginals=False, map_=True))):
            if a.variants is not None and name not in a.variants:
                continue
            plan.extra_mode = extra
            out = plan.alloc_outputs(rows, **outs)
            for _ in range(3):
                plan.run(d, rows, 0, rows, out)
            bound = plan.bind(d, rows, 0, rows, out)  # prepared launch (what bench.py times)
            for _ in range(3):
                bound.run()
            t = HipTimer()
            t.start()
            for _ in range(a.reps):
                bound.run()
            us = t.stop_ms() * 1e3 / a.reps
            t.start()
            for _ in range(a.reps):
                plan.run(d, rows, 0, rows, out)
            us_unbound = t.stop_ms() * 1e3 / a.reps
            import time as _t
            torch.cuda.synchronize()
            c0 = _t.perf_counter()
            for _ in range(a.reps):
                bound.run()
            cpu_us = (_t.perf_counter() - c0) * 1e6 / a.reps  # host cost per launch (GPU may lag behind)
            c0 = _t.perf_counter()
            for _ in range(a.reps):
                N.lib().pgm_version()
            ctypes_us = (_t.perf_counter() - c0) * 1e6 / a.reps  # bare ctypes call, for comparison
            torch.cuda.synchronize()
            bpr = plan.algorithmic_bytes_per_row(marginals=outs.get("marginals", False), map_=outs.get("map_", False))
            print(json.dumps({"rows": rows, "variant": name, "kernel_us": us, "rows_per_s": rows / us * 1e6,
                              "GBps": bpr * rows / us / 1e3, "bytes_per_row": bpr, "unbound_us": us_unbound, "host_us_per_launch": cpu_us, "ctypes_call_us": ctypes_us}),
                  flush=True)
        plan.extra_mode = 0
        if a.variants is None or "compact_codes" in a.variants:
            # same rows, only the plan's evidence columns (a [7, rows] matrix instead of [1035, rows])
            used = plan.ev_used
            pos_obs = {v: i for i, v in enumerate(obs)}
            d2 = upload_codes(np.ascontiguousarray(np.tile(ev[[pos_obs[v] for v in used]], (1, rep))[:, :rows]))
            plan2 = PatternPlan(m, missing, used, {v: i for i, v in enumerate(used)})
            for name, outs in (("compact_codes", dict(marginals=True)), ("compact_map_only", dict(marginals=False, map_=True))):
                out = plan2.alloc_outputs(rows, **outs)
                for _ in range(3):
                    plan2.run(d2, rows, 0, rows, out)
                t = HipTimer()
                t.start()
                for _ in range(a.reps):
                    plan2.run(d2, rows, 0, rows, out)
                us = t.stop_ms() * 1e3 / a.reps
                bpr = plan2.algorithmic_bytes_per_row(marginals=outs.get("marginals", False), map_=outs.get("map_", False))
                print(json.dumps({"rows": rows, "variant": name, "kernel_us": us, "rows_per_s": rows / us * 1e6,
                                  "GBps": bpr * rows / us / 1e3, "bytes_per_row": bpr}), flush=True)
            del d2
        del d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
