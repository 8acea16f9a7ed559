#!/usr/bin/env python3
"""The C2 program (munin, the reference's 20-row pattern): each step's note, grid and time replayed alone
(Program.time_steps), and the whole program as graph and as AQL chain.  Profiling aid."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")))
    q = g["variables"]
    ve = VariableElimination(get_example_model("munin"))
    ve.query(q, g["rows"][0]["evidence"], show_progress=False)
    torch.cuda.synchronize()
    runner, = ve._compiled.values()
    (prog, *_), = runner.plan.__dict__["_progs"].values()
    steps = prog.time_steps(reps=20)
    tot = 0.0
    for us, note in steps:
        tot += us
        print(f"{us:7.2f} us  {note[:150]}")
    print(f"{len(steps)} steps, {tot:.1f} us summed; direct: {prog.direct_note}")


if __name__ == "__main__":
    main()
