#!/usr/bin/env python3
"""C1 alarm query patterns (bench.py bench_c1), run twice through compiled plans: per pattern the plan kind,
and any error; with --chain the levelled-batch lowering (PGM_BATCH_LEVELS=1) too, results compared with
the per-level launches (diagnostic)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(chain):
    import numpy as np

    import pgmpy_amd.program as P
    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    P.LEVEL_CHAIN = chain
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
    res, bad = [], []
    for rep in range(3):
        for i, (q, e) in enumerate(pats):
            try:
                r = ve.query(q, e, show_progress=False)
                if rep == 2:
                    res.append(np.asarray(r.values).ravel())
            except Exception as ex:  # noqa: BLE001
                runner = [rr for k, rr in ve._compiled.items() if list(k[0]) == q][0]
                pl = runner.plan
                bad.append((rep, i, type(ex).__name__, str(ex)[:80], pl.kind, len(pl.ev_used),
                            [n for n in getattr(pl, "_progs", {}).values()][0][0].notes[:3] if getattr(pl, "_progs", None) else None))
                if rep == 2:
                    res.append(None)
    return res, bad


def main():
    off, bad0 = run(False)
    print("per-level launches: errors", bad0[:5], flush=True)
    if "--chain" in sys.argv:
        on, bad1 = run(True)
        print("levelled chain: errors", bad1[:5], flush=True)
        import numpy as np

        diff = [i for i, (a, b) in enumerate(zip(off, on)) if a is None or b is None or not np.allclose(a, b, rtol=1e-12)]
        print("patterns differing:", diff)
    sys.exit(1 if bad0 else 0)


if __name__ == "__main__":
    main()
