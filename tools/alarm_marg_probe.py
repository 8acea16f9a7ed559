#!/usr/bin/env python3
"""Per-query time of the alarm golden patterns with joint=False vs joint=True, and the plan kinds."""
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from tests.goldens import load_json

    pats = load_json("alarm_queries.json")["patterns"]
    for joint in (True, False):
        ve = VariableElimination(get_example_model("alarm"))
        for p in pats:
            ve.query(p["variables"], p["evidence"], joint=joint, show_progress=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            for p in pats:
                ve.query(p["variables"], p["evidence"], joint=joint, show_progress=False)
        dt = (time.perf_counter() - t0) / (20 * len(pats))
        kinds = collections.Counter(rn.plan.kind for rn in ve._compiled.values())
        per = collections.defaultdict(list)
        for p in pats[:50]:
            t1 = time.perf_counter()
            for _ in range(20):
                ve.query(p["variables"], p["evidence"], joint=joint, show_progress=False)
            key = (tuple(p["variables"]), tuple(sorted(p["evidence"], key=str)), joint)
            per[ve._compiled[key].plan.kind].append((time.perf_counter() - t1) / 20 * 1e6)
        print(f"joint={joint}: {dt * 1e6:.1f} us/query, plan kinds {dict(kinds)}, "
              + ", ".join(f"{k}: median {sorted(v)[len(v) // 2]:.1f} us" for k, v in per.items()), flush=True)


if __name__ == "__main__":
    main()
