"""C1 warm-query latency breakdown: alarm, 50 seeded patterns (bench.py --workload c1), cProfile of
the warm loop.  python tools/c1_profile.py"""
import cProfile
import os
import pstats
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    t0 = time.perf_counter()
    for _ in range(10):
        for q, e in pats:
            ve.query(q, e, show_progress=False)
    torch.cuda.synchronize()
    print("warm ms/query", (time.perf_counter() - t0) / 500 * 1e3, flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(4):
        for q, e in pats:
            ve.query(q, e, show_progress=False)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
