#!/usr/bin/env python3
"""C1-shaped alarm queries in blocks: per-block time per query, live Python objects and the types that
grow (finds per-query leaks that make long runs slower)."""
import collections
import gc
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
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
        q, e = pick[:3], pick[3:]
        pats.append((q, {v: m.states[v][codes[pos[v], r]] for v in e}))
    ve = VariableElimination(m)
    for q, e in pats:
        ve.query(q, e, show_progress=False)
    torch.cuda.synchronize()
    prev = None
    for blk in range(8):
        gc.collect()
        counts = collections.Counter(type(o).__name__ for o in gc.get_objects())
        t0 = time.perf_counter()
        for _ in range(5):
            for q, e in pats:
                ve.query(q, e, show_progress=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 250
        grow = [] if prev is None else sorted(((counts[k] - prev.get(k, 0), k) for k in counts), reverse=True)[:6]
        print(f"block {blk}: {dt * 1e6:.1f} us/query, objects {sum(counts.values())}, gc counts {gc.get_count()}, grew {grow}",
              flush=True)
        prev = counts


if __name__ == "__main__":
    main()
