#!/usr/bin/env python3
"""Where a compiled single query's time goes, C1 (alarm, the reference's 50 golden patterns) and C2 (munin,
the 20 golden rows): the whole ve.query, the AQL chains alone (each program's run_direct: ctypes call +
GPU + spin wait) and the Python part alone (run_direct replaced by a no-op); medians over N rounds, plus a
cProfile of the Python part.

    python3 tools/query_split.py [N]"""
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def split(name, ve, calls, n):
    import torch

    for q, e in calls * 3:
        ve.query(q, e, show_progress=False)
    torch.cuda.synchronize()
    progs = [h[0] for rn in ve._compiled.values() for h in rn.plan.__dict__.get("_q1", {}).values()]

    def per_query(fn):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            for c in calls:
                fn(c)
            ts.append((time.perf_counter() - t0) / len(calls))
        return statistics.median(ts) * 1e6

    out = {"config": name, "programs": len(progs),
           "whole_us": per_query(lambda c: ve.query(c[0], c[1], show_progress=False))}
    # the chains alone, in the same round-robin order as the queries (one program per pattern)
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        for p in progs:
            p.run_direct()
        ts.append((time.perf_counter() - t0) / len(progs))
    out["chains_us"] = statistics.median(ts) * 1e6
    # the Python part alone: every chain made a no-op (the programs' run_direct, and the bound fast
    # callers of repeat calls, QueryRunner.bytes_caller, which run the chain themselves)
    real = [p.run_direct for p in progs]
    fast = ve.__dict__.get("_fast", {})
    real_fast = {k: f.fast for k, f in fast.items()}
    for f in fast.values():
        if f.fast:
            res = f.fast.keep[1][f.runner.key].array.reshape(-1)
            f.fast = lambda codes, r=res: r.copy()
    for p in progs:
        p.run_direct = lambda: None
    try:
        out["python_us"] = per_query(lambda c: ve.query(c[0], c[1], show_progress=False))
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(max(1, n // 4)):
            for q, e in calls:
                ve.query(q, e, show_progress=False)
        pr.disable()
    finally:
        for p, r in zip(progs, real):
            p.run_direct = r
        for k, f in fast.items():
            f.fast = real_fast[k]
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(22)
    print(json.dumps(out, indent=1))
    print(s.getvalue())
    return out


def main(n=200):
    n = int(n)
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    g1 = json.load(open(os.path.join(ROOT, "tests", "golden", "alarm_queries.json")))
    ve1 = VariableElimination(get_example_model("alarm"))
    r1 = split("c1", ve1, [(p["variables"], p["evidence"]) for p in g1["patterns"]], n)
    g2 = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")))
    ve2 = VariableElimination(get_example_model("munin"))
    r2 = split("c2", ve2, [(g2["variables"], r["evidence"]) for r in g2["rows"]], n)
    print(json.dumps({"c1": r1, "c2": r2}))


if __name__ == "__main__":
    main(*sys.argv[1:])
