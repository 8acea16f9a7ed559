#!/usr/bin/env python3
"""Diagnostic: C1 pattern 4 (a steps plan) queried repeatedly on its own; device codes buffer and error
flag after each query (r03g: the second query of a steps plan raised the gather's out-of-range flag)."""
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
    q, e = pats[4]
    ve = VariableElimination(m)
    for k in range(4):
        try:
            r = ve.query(q, e, show_progress=False)
            ok = "ok"
        except IndexError as ex:
            ok = str(ex)
        runner = list(ve._compiled.values())[0]
        pl = runner.plan
        prog, cbuf, perr, bufs, cols_dev, host = list(pl._progs.values())[0]
        torch.cuda.synchronize()
        print(k, ok, "ev_used", pl.ev_used, "sel", getattr(pl, "_ev_sel", None), "host codes", host["codes"].numpy().ravel().tolist(),
              "dev codes", cbuf.cpu().numpy().ravel().tolist(), "perr", int(perr.item()), "host err", int(host["err"].numpy()[0]),
              "cards", [pl.card[v] for v in pl.ev_used], flush=True)
    print("notes", prog.notes[:6])


if __name__ == "__main__":
    main()
