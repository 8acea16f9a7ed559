#!/usr/bin/env python3
"""Microbenchmarks of the generic kernels on BP-like shapes (HIP-event timing).

    python tools/micro_kernels.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps=10):
    from bench import HipTimer

    fn()
    t = HipTimer()
    t.start()
    for _ in range(reps):
        fn()
    return t.stop_ms() * 1e3 / reps


def main():
    import numpy as np

    from pgmpy_amd import engine as E

    rng = np.random.default_rng(0)
    R = 10000
    for clique in ([4, 4, 4, 8], [8, 8, 8, 63], [2] * 9):
        labels = [f"v{i}" for i in range(len(clique))]
        n = int(np.prod(clique))
        pot = E.to_device(rng.random(clique))
        ops = [(pot, labels)]
        for k in range(7):
            l = labels[k % len(labels)]
            ops.append((E.to_device(rng.random((clique[k % len(labels)], R))), [l, "R"]))
        for nops in (2, 4, 8):
            us = timeit(lambda: E.product_n(ops[:nops], labels + ["R"]))
            gb = 8 * n * R / us / 1e3
            print(json.dumps({"kernel": "product_n", "clique": clique, "ops": nops, "us": us, "write_GBps": gb}))
        B = E.product_n(ops[:2], labels + ["R"])
        us = timeit(lambda: E.contract(B, labels + ["R"], None, None, [labels[0], "R"], reduce="sum", combine="copy"))
        print(json.dumps({"kernel": "marg_to_first", "clique": clique, "us": us, "read_GBps": 8 * n * R / us / 1e3}))
        us = timeit(lambda: E.contract(B, labels + ["R"], None, None, [labels[-1], "R"], reduce="sum", combine="copy"))
        print(json.dumps({"kernel": "marg_to_last", "clique": clique, "us": us, "read_GBps": 8 * n * R / us / 1e3}))
        S = E.contract(B, labels + ["R"], None, None, [labels[1], "R"], reduce="sum", combine="copy")
        us = timeit(lambda: E.contract(B, labels + ["R"], S, [labels[1], "R"], labels + ["R"], combine="mul", out=B))
        print(json.dumps({"kernel": "update_inplace", "clique": clique, "us": us, "rw_GBps": 16 * n * R / us / 1e3}))


if __name__ == "__main__":
    main()
