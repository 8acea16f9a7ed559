#!/usr/bin/env python3
"""Time every step of a compiled program alone and list the slowest (profiling aid).

    python tools/program_steps.py c4 [rows]      # batched BP schedule on pathfinder
    python tools/program_steps.py c2             # munin C2 query plan
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "c4"
    if what == "c4":
        from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
        from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
        from pgmpy_amd.utils import get_example_model

        n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
        m = get_example_model("pathfinder")
        bjt = BatchedJunctionTree(junction_tree_from_model(m))
        leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
        sch = bjt.schedule(n, leaves, graph=False, marginals=False)
        sch.codes.zero_()  # valid evidence (state 0 everywhere): the findings kernels flag bad codes
        prog = sch.prog
    else:
        import random

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
        ve.query(q, ev, show_progress=False)
        runner, = ve._compiled.values()
        (prog, *_), = runner.plan._progs.values()
    res = prog.time_steps()
    tot = sum(us for us, _ in res)
    if not prog._levels:
        job_detail(prog, res)
    import torch

    prog.run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        prog.run()
    b.record()
    torch.cuda.synchronize()
    stream_ms = a.elapsed_time(b) / 10
    prog.capture()
    prog.run()
    torch.cuda.synchronize()
    a.record(prog._stream)
    for _ in range(10):
        prog.run(prog._stream)
    b.record(prog._stream)
    torch.cuda.synchronize()
    print(f"{len(res)} steps, {tot / 1e3:.2f} ms summed; whole program back to back: stream launches "
          f"{stream_ms:.2f} ms, graph replay {a.elapsed_time(b) / 10:.2f} ms")
    if prog._recs:
        import collections

        big, small = collections.Counter(), collections.Counter()
        for r in prog._recs:
            (big if r.job is None else small)[r.level] += 1
        print("levels:", prog.n_levels, " unbatched launches per level:",
              [big[lv] for lv in range(prog.n_levels)], " batched jobs per level:",
              [small[lv] for lv in range(prog.n_levels)])
    if os.environ.get("LEVELS") and prog._recs:
        tot_b = 0
        for lv in range(prog.n_levels):
            idx = [i for i, l in enumerate(prog.step_levels) if l == lv]
            us_l = sum(res[i][0] for i in idx)
            b_l = sum(prog.step_bytes[i] for i in idx)
            tot_b += b_l
            print(f"-- level {lv}: {len(idx)} launches, {us_l:.1f} us, {b_l / 1e6:.1f} MB, "
                  f"{b_l / max(us_l, 1e-9) / 1e3:.0f} GB/s")
            for i in idx:
                us, note = res[i]
                print(f"   {us:8.1f} us {prog.step_bytes[i] / 1e6:9.1f} MB {prog.step_bytes[i] / max(us, 1e-9) / 1e3:6.0f} GB/s"
                      f"  {note[:120]}")
        print(f"total algorithmic bytes of the steps: {tot_b / 1e6:.1f} MB")
    top = int(os.environ.get("TOP", "25"))
    for us, note in sorted(res, key=lambda r: -r[0])[:top]:
        print(f"{us:9.1f} us  {note[:220] if len(sys.argv) < 4 else note}")


def job_detail(prog, res, top=6):
    """Plain program: the jobs of the slowest steps (_plain_recs grouped by launch, in launch order),
    each with the bytes its footprint spans (hazard.py)."""
    units = sorted({r.step for r in prog._plain_recs})
    if len(units) != len(res):
        return
    by = {}
    for r in prog._plain_recs:
        by.setdefault(r.step, []).append(r)
    for i in sorted(range(len(res)), key=lambda i: -res[i][0])[:top]:
        jobs = by[units[i]]
        print(f"{res[i][0]:8.1f} us  {res[i][1][:60]}")
        for r in sorted(jobs, key=lambda r: -sum(hi - lo for lo, hi, _ in r.foot or []))[:8]:
            print(f"           {sum(hi - lo for lo, hi, _ in r.foot or []) / 1e6:8.3f} MB  {r.note[:110]}")


if __name__ == "__main__":
    main()
