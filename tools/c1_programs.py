#!/usr/bin/env python3
"""C1's compiled programs (alarm, the reference's 50 golden patterns): launches per AQL chain and each
step's note, and each program's steps replayed alone (Program.time_steps) for the first few."""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "alarm_queries.json")))
    ve = VariableElimination(get_example_model("alarm"))
    for p in g["patterns"]:
        ve.query(p["variables"], p["evidence"], show_progress=False)
    torch.cuda.synchronize()
    hist = collections.Counter()
    shown = 0
    for rn in ve._compiled.values():
        for prog, _ in rn.plan.__dict__.get("_q1", {}).values():
            hist[len(prog._direct or ())] += 1
            if shown < 4:
                shown += 1
                print(prog.direct_note)
                for us, note in prog.time_steps(reps=20):
                    print(f"  {us:6.2f} us  {note[:110]}")
    print("launches per chain -> programs:", dict(sorted(hist.items())))


if __name__ == "__main__":
    main()
