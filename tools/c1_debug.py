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
    for i in (4, 9, 4, 9):
        q, e = pats[i]
        try:
            ve.query(q, e, show_progress=False)
            ok = "ok"
        except IndexError as ex:
            ok = str(ex)
        key = [k for k in ve._compiled if list(k[0]) == q][0]
        pl = ve._compiled[key].plan
        prog, cbuf, perr, bufs, cols_dev, host = list(pl._progs.values())[0]
        torch.cuda.synchronize()
        print(i, ok, "plan", id(pl), "ev_used", pl.ev_used, "codes", [pl.card[v] for v in pl.ev_used],
              "host", host["codes"].numpy().ravel().tolist(), "dev", cbuf.cpu().numpy().ravel().tolist(),
              "perr", int(perr.item()), "cbuf ptr", hex(cbuf.data_ptr()), "perr ptr", hex(perr.data_ptr()), flush=True)
    q, e = pats[4]
    key = [k for k in ve._compiled if list(k[0]) == q][0]
    pl = ve._compiled[key].plan
    prog, cbuf, perr, bufs, cols_dev, host = list(pl._progs.values())[0]
    s = N.stream_handle()
    for j, (step, note) in enumerate(zip(prog._steps, prog.notes)):
        step(s)
        torch.cuda.synchronize()
        print("step", j, note[:90], "perr", int(perr.item()), flush=True)


if __name__ == "__main__":
    main()
