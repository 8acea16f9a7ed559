#!/usr/bin/env python3
"""Host time of the C2 query's graph launch (pgm_graph_launch) against its completion: is the single
query bound by the host's submission of the graph's kernel nodes?  python tools/c2_host_launch.py"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("munin")
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    roots = sorted(v for v in m.nodes() if m.in_degree(v) == 0)
    rng = random.Random(100000)
    E = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    ev = {v: m.states[v][0] for v in E}
    ve = VariableElimination(m)
    for _ in range(5):
        ve.query(q, ev, show_progress=False)
    runner, = ve._compiled.values()
    (prog, *_), = runner.plan._progs.values()
    L = N.lib()
    s = N.stream_handle()
    torch.cuda.synchronize()
    launch, total = [], []
    for _ in range(50):
        t0 = time.perf_counter()
        prog.run()
        t1 = time.perf_counter()
        N.check(L.pgm_stream_sync_spin(s))
        t2 = time.perf_counter()
        launch.append((t1 - t0) * 1e6)
        total.append((t2 - t0) * 1e6)
    launch.sort()
    total.sort()
    q0 = []
    for _ in range(50):
        t0 = time.perf_counter()
        ve.query(q, ev, show_progress=False)
        q0.append((time.perf_counter() - t0) * 1e6)
    q0.sort()
    print(f"steps {len(prog)}: graph launch host median {launch[25]:.1f} us, launch -> done median {total[25]:.1f} us, "
          f"whole query() median {q0[25]:.1f} us")


if __name__ == "__main__":
    main()
