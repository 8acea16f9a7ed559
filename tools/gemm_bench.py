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
        import torch

        for name, fn in (("gemm", lambda: L.pgm_gemm(ctypes.byref(d), N.ptr(A), N.ptr(B), N.ptr(Cg), N.stream_handle())),
                         ("generic", lambda: E.contract(A, la, B, lb, keep, reduce="sum", combine="mul")),
                         # ceiling reference only (not used by the engine): the vendor FP64 GEMM on plain layouts
                         ("rocblas_ref", lambda: torch.bmm(A, B))):
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
        # the other unit-stride layouts: A stored m-innermost, B stored k-innermost
        At = E.to_device(np.ascontiguousarray(E.to_host(A).transpose(0, 2, 1)))  # [b, k, m]
        Bt = E.to_device(np.ascontiguousarray(E.to_host(B).transpose(0, 2, 1)))  # [b, n, k]
        d2, table2, C2 = E.prepare_gemm(At, ["b", "k", "m"], Bt, ["b", "n", "k"], keep, (["b"], ["m"], ["n"], ["k"]))
        fn = lambda: L.pgm_gemm(ctypes.byref(d2), N.ptr(At), N.ptr(Bt), N.ptr(C2), N.stream_handle())  # noqa: E731
        fn()
        t = HipTimer()
        t.start()
        for _ in range(5):
            fn()
        us = t.stop_ms() * 1e3 / 5
        res["gemm_mk_nk_us"] = us
        res["gemm_mk_nk_TFLOPs"] = 2 * nb * m * n * k / us / 1e6
        res["mk_nk_max_rel_diff"] = float(np.max(np.abs(E.to_host(C2) - R) / np.abs(R)))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
