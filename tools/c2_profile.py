"""C2 warm-query breakdown: wall per query, the compiled program's graph replay alone (HIP events),
and a cProfile of the warm loop.  python tools/c2_profile.py"""
import cProfile
import ctypes
import os
import pstats
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    roots = sorted(n for n in m.nodes() if m.in_degree(n) == 0)
    rng = random.Random(100000)
    E = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    codes, nodes = forward_sample_codes(m, 1, seed=0)
    ev = {v: m.states[v][codes[nodes.index(v), 0]] for v in E}
    ve = VariableElimination(m)
    for _ in range(3):
        ve.query(q, ev, show_progress=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        ve.query(q, ev, show_progress=False)
    torch.cuda.synchronize()
    print("warm ms/query", (time.perf_counter() - t0) / 20 * 1e3, flush=True)
    runner, = ve._compiled.values()
    plan = runner.plan
    (prog, cbuf, perr, bufs, cols_dev, _host), = plan._progs.values()
    L = N.lib()
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    N.check(L.pgm_event_create(ctypes.byref(a)))
    N.check(L.pgm_event_create(ctypes.byref(b)))
    s = N.stream_handle()
    N.check(L.pgm_event_record(a, s))
    for _ in range(20):
        prog.run()
    N.check(L.pgm_event_record(b, s))
    ms = ctypes.c_float()
    N.check(L.pgm_event_elapsed_ms(a, b, ctypes.byref(ms)))
    print("graph replay ms", ms.value / 20, flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        ve.query(q, ev, show_progress=False)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
