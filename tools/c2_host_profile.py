#!/usr/bin/env python3
"""Host-side profile of the C2 query path on the GPU (profiling aid): cProfile over repeated
VariableElimination.query calls of bench.py's munin C2 pattern, top functions by own time.

    python3 tools/c2_host_profile.py [N]"""
import cProfile
import os
import pstats
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    roots = sorted(v for v in m.nodes() if m.in_degree(v) == 0)
    rng = random.Random(100000)
    ev_vars = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    codes, nodes = forward_sample_codes(m, 1, seed=0)
    evidence = {v: m.states[v][codes[nodes.index(v), 0]] for v in ev_vars}
    ve = VariableElimination(m)
    for _ in range(50):
        ve.query(q, evidence, show_progress=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        ve.query(q, evidence, show_progress=False)
    print(f"{n} queries, {(time.perf_counter() - t0) / n * 1e3:.4f} ms each (no profiler)")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        ve.query(q, evidence, show_progress=False)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)




def split():
    """Where one query's wall time goes: the Python part before the launch, the graph launch call on
    the host, and the wait for the GPU (spin), averaged over N queries of the C2 pattern."""
    import ctypes

    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    n = 2000
    m = get_example_model("munin")
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    roots = sorted(v for v in m.nodes() if m.in_degree(v) == 0)
    rng = random.Random(100000)
    ev_vars = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    codes, nodes = forward_sample_codes(m, 1, seed=0)
    evidence = {v: m.states[v][codes[nodes.index(v), 0]] for v in ev_vars}
    ve = VariableElimination(m)
    for _ in range(50):
        ve.query(q, evidence, show_progress=False)
    runner, = ve._compiled.values()
    plan = runner.plan
    prog = plan._steps_program(1, frozenset(["marg"]), host_io=True)[0]
    L = N.lib()
    s = N.stream_handle()
    torch.cuda.synchronize()
    tl = tw = 0.0
    for _ in range(n):
        t0 = time.perf_counter()
        prog.run()
        t1 = time.perf_counter()
        N.check(L.pgm_stream_sync_spin(s), "spin")
        t2 = time.perf_counter()
        tl += t1 - t0
        tw += t2 - t1
    t0 = time.perf_counter()
    for _ in range(n):
        ve.query(q, evidence, show_progress=False)
    tq = time.perf_counter() - t0
    print(f"query {tq / n * 1e6:.1f} us; graph launch call {tl / n * 1e6:.1f} us; launch->done wait {tw / n * 1e6:.1f} us; "
          f"rest (python, codes, result) {(tq - tl - tw) / n * 1e6:.1f} us")


if __name__ == "__main__":
    split() if sys.argv[1:2] == ["split"] else main()
