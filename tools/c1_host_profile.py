#!/usr/bin/env python3
"""cProfile of 1,000 C1-shaped alarm queries (after compiling their plans): where the host time of a
compiled single query goes."""
import cProfile
import io
import os
import pstats
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import gc

    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("alarm")
    nodes_sorted = sorted(m.nodes())
    rng = random.Random(1)
    codes, nodes = forward_sample_codes(m, 50, seed=1)
    pos = {v: i for i, v in enumerate(nodes)}
    pats = []
    for r in range(50):
        pick = rng.sample(nodes_sorted, 8)
        pats.append((pick[:3], {v: m.states[v][codes[pos[v], r]] for v in pick[3:]}))
    ve = VariableElimination(m)
    for q, e in pats:
        ve.query(q, e, show_progress=False)
    torch.cuda.synchronize()
    gc.collect()
    t0 = time.perf_counter()
    for _ in range(20):
        for q, e in pats:
            ve.query(q, e, show_progress=False)
    print("plain us/query", (time.perf_counter() - t0) / 1000 * 1e6)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        for q, e in pats:
            ve.query(q, e, show_progress=False)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
