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
    ve.query(*pats[4], show_progress=False)
    for i in range(50):
        if i == 4:
            continue
        q, e = pats[i]
        ve.query(q, e, show_progress=False)
        key = [k for k in ve._compiled if list(k[0]) == q][0]
        pl = ve._compiled[key].plan
        try:
            ve.query(*pats[4], show_progress=False)
            ok = "ok"
        except IndexError as ex:
            ok = str(ex)
        print(i, pl.kind, pl.variables, pl.ev_used, "n_comp", pl.n_comp, "-> pattern 4:", ok, flush=True)
        if ok != "ok":
            print("culprit", i, pl.describe(), flush=True)
            break


if __name__ == "__main__":
    main()
