#!/usr/bin/env python3
"""C1 / C2 query latency under n-ary fusion settings (r06 A/B aid): for each (budget, max_red) the
compiled C2 pattern's AQL chain (launches, us per run) and the whole query, and C1's 50 patterns.

    python3 tools/fuse_sweep.py budget:max_red[:crit] [...]    (0:0 = no fusion; crit 0/1, default 1)"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(*settings):
    import torch

    import pgmpy_amd.inference.contraction as C
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    g2 = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")))
    g1 = json.load(open(os.path.join(ROOT, "tests", "golden", "alarm_queries.json")))
    munin, alarm = get_example_model("munin"), get_example_model("alarm")
    q2, rows2 = g2["variables"], [r["evidence"] for r in g2["rows"]]
    pats = [(p["variables"], p["evidence"]) for p in g1["patterns"]]
    res = []
    for st in settings:
        parts = [int(x) for x in st.split(":")]
        b, r = parts[0], parts[1]
        C.FUSE_CRITICAL_ONLY = bool(parts[2]) if len(parts) > 2 else True
        C.FUSE = b > 0
        if b:
            C.FUSE_BUDGET, C.FUSE_MAX_RED = b, r
        C._PATHS.clear()
        ve2, ve1 = VariableElimination(munin), VariableElimination(alarm)
        for k in range(60):
            ve2.query(q2, rows2[k % 20], show_progress=False)
        for q, e in pats:
            ve1.query(q, e, show_progress=False)
        torch.cuda.synchronize()
        runner, = ve2._compiled.values()
        prog = runner.plan.__dict__["_q1"]["joint"][0]
        ts = []
        for _ in range(500):
            t0 = time.perf_counter()
            prog.run_direct()
            ts.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        for k in range(1000):
            ve2.query(q2, rows2[k % 20], show_progress=False)
        c2 = (time.perf_counter() - t0) / 1000
        t0 = time.perf_counter()
        for _ in range(10):
            for q, e in pats:
                ve1.query(q, e, show_progress=False)
        c1 = (time.perf_counter() - t0) / (10 * len(pats))
        res.append({"budget": b, "max_red": r, "crit": C.FUSE_CRITICAL_ONLY, "c2_launches": len(prog._direct) if prog._direct else None,
                    "c2_chain_us": statistics.median(ts) * 1e6, "c2_us": c2 * 1e6, "c1_us": c1 * 1e6,
                    "levels": runner.plan.path_stats(1).get("levels")})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
