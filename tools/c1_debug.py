#!/usr/bin/env python3
"""Diagnostic: C1 steps plans queried in turn (pattern 4, then 9, then 4 again); after each query the
plan object, codes, device codes buffer and error flag; then pattern 4's program replayed step by step
(no graph) to find the step that raises the flag (r03g: the second query of a steps plan raised it once
another steps plan had been compiled)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("alarm")
    nodes_sorted = sorted(m.nodes())
    rng = random.Random(1)
    codes, nodes = forward_sample_codes(m, 50, seed=1)
    pos = {v: i for i, v in enumerate(nodes)}
    pats = []
    for r in range(50):
        pick = rng.sample(nodes_sorted, 8)
        pats.append((pick[:3], {v: m.states[v][codes[pos[v], r]] for v in pick[3:]}))
    ve = VariableElimination(m)
    s = N.stream_handle()
    for rep in range(2):
        for i, (q, e) in enumerate(pats):
            try:
                ve.query(q, e, show_progress=False)
                continue
            except IndexError as ex:
                ok = str(ex)
            key = [k for k in ve._compiled if list(k[0]) == q][0]
            pl = ve._compiled[key].plan
            prog, cbuf, perr, bufs, cols_dev, host = list(pl._progs.values())[0]
            torch.cuda.synchronize()
            print("rep", rep, "pattern", i, ok, pl.ev_used, [pl.card[v] for v in pl.ev_used], "dev codes",
                  cbuf.cpu().numpy().ravel().tolist(), "perr", int(perr.item()), flush=True)
            for j, (step, note) in enumerate(zip(prog._steps, prog.notes)):
                step(s)
                torch.cuda.synchronize()
                print("  step", j, note[:100], "perr", int(perr.item()), flush=True)
            print("graph replay:", flush=True)
            prog.run()
            torch.cuda.synchronize()
            print("  perr after graph", int(perr.item()), flush=True)
            return


if __name__ == "__main__":
    main()
