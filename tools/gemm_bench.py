#!/usr/bin/env python3
"""FP64 MFMA dense steps (pgm_gemm) vs the generic fused contraction on C2's largest greedy steps.

    python tools/gemm_bench.py
One JSON line per shape: us and TFLOP/s for both paths (HIP events, same stream)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [  # (batch, M, N, K) of the munin C2 query's largest pairwise steps
    (1, 3000, 12000, 112), (500, 100, 576, 125), (5, 384, 800, 700), (80, 16, 480, 750), (80, 80, 480, 144),
    (1, 4096, 4096, 512),
]


def main():
    import numpy as np

    import ctypes

    from bench import HipTimer
    from pgmpy_amd import _native as N
    from pgmpy_amd import engine as E

    rng = np.random.default_rng(0)
    for nb, m, n, k in SHAPES:
        A = E.to_device(rng.random((nb, m, k)))
        B = E.to_device(rng.random((nb, k, n)))
        la, lb, keep = ["b", "m", "k"], ["b", "k", "n"], ["b", "m", "n"]
        res = {"batch": nb, "M": m, "N": n, "K": k}
        d, table, Cg = E.prepare_gemm(A, la, B, lb, keep, (["b"], ["m"], ["n"], ["k"]))  # prebuilt, as in programs
        L = N.lib()
        for name, fn in (("gemm", lambda: L.pgm_gemm(ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(Cg), N.stream_handle())),
                         ("generic", lambda: E.contract(A, la, B, lb, keep, reduce="sum", combine="mul"))):
            fn()
            reps = 5
            t = HipTimer()
            t.start()
            for _ in range(reps):
                fn()
            us = t.stop_ms() * 1e3 / reps
            res[f"{name}_us"] = us
            res[f"{name}_TFLOPs"] = 2 * nb * m * n * k / us / 1e6
        C = E.to_host(E.pair_gemm(A, la, B, lb, keep, force=True))
        R = E.to_host(E.contract(A, la, B, lb, keep, reduce="sum", combine="mul"))
        res["max_rel_diff"] = float(np.max(np.abs(C - R) / np.abs(R)))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
