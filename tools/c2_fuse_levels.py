#!/usr/bin/env python3
"""C2's compiled program with and without n-ary fusion (r06 profiling aid): per level of the planned path,
the jobs (kind, outputs, reduction entries per output, inputs), and each lowered step's time replayed
alone (Program.time_steps).

    python3 tools/c2_fuse_levels.py [budget [max_red]]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(budget=None, max_red=None):
    import torch

    import pgmpy_amd.inference.contraction as C
    from pgmpy_amd import engine as E
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    if budget:
        C.FUSE_BUDGET = int(budget)
    if max_red:
        C.FUSE_MAX_RED = int(max_red)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")))
    q = g["variables"]
    for fuse in ((True,) if os.environ.get("FUSED_ONLY") else (True, False)):
        C.FUSE = fuse
        C._PATHS.clear()
        ve = VariableElimination(get_example_model("munin"))
        ve.query(q, g["rows"][0]["evidence"], show_progress=False)
        torch.cuda.synchronize()
        runner, = ve._compiled.values()
        plan = runner.plan
        # the planned path's levels (as contract_factors records them)
        labels, dims = [], dict(plan.card)
        dims[E.ROW] = 1
        for vars_, _ in plan.factors:
            ls = [v for v in vars_ if v not in plan.evidence_vars]
            if any(v in plan.evidence_vars for v in vars_):
                ls = ls + [E.ROW]
            labels.append(ls)
        steps, final_id, levels = C.compiled_path(labels, plan.variables + [E.ROW], dims, fuse=fuse)
        lab = {i: list(dict.fromkeys(ls)) for i, ls in enumerate(labels)}
        print(f"== fuse={fuse} levels={len(levels)} steps={len(steps)}")
        for li, lvl in enumerate(levels):
            jobs = []
            for k in lvl:
                st = steps[k][0]
                ins, keep = st[1:-2], st[-2]
                space = list(dict.fromkeys(l for i in ins for l in lab[i]))
                n_out = C._size(keep, dims)
                jobs.append((st[0], n_out, C._size(space, dims) // max(1, n_out), len(ins)))
                lab[st[-1]] = keep
            big = sorted(jobs, key=lambda j: -j[1] * j[2])[:3]
            work = sum(j[1] * j[2] * j[3] for j in jobs)
            print(f"  level {li:2d}: {len(jobs):3d} jobs, work {work:9d}, heaviest {big}")
        prog = plan.__dict__["_q1"]["joint"][0]
        tot = 0.0
        for i, (us, note) in enumerate(prog.time_steps(reps=20)):
            tot += us
            print(f"  {us:7.2f} us  {note[:100]}")
            if us > 4.5 and os.environ.get("JOB_TIMES"):  # the slowest jobs of a slow launch, each alone
                for t, kind, desc in sorted(prog.time_step_jobs(i), key=lambda r: -r[0])[:4]:
                    print(f"      {t:6.2f} us  {kind} {desc}")
        print(f"  {tot:.1f} us summed; {prog.direct_note}")
        dump = os.environ.get("DUMP_SRC")
        if dump and fuse:  # each launch's generated source (compile it with hipcc to read its resources)
            import ctypes

            from pgmpy_amd import _native as N

            os.makedirs(dump, exist_ok=True)
            L, buf = N.lib(), ctypes.create_string_buffer(1 << 22)
            for i, st in enumerate(prog._steps):
                for j, b in enumerate(getattr(st, "bounds", ())):
                    n = L.pgm_pm_bound_source(b, buf, len(buf))
                    if n > 0:
                        with open(os.path.join(dump, f"step_{i}_{j}.hip"), "w") as f:
                            f.write(buf.value.decode())


if __name__ == "__main__":
    main(*sys.argv[1:])
