#!/usr/bin/env python3
"""Print and time the widest collect products of the C4 schedule (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from bench import HipTimer
    from pgmpy_amd import engine as E
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model

    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    n = 2000
    sizes = sorted(bjt.sizes.items(), key=lambda kv: -kv[1])[:5]
    print("largest cliques", [(len(c), s) for c, s in sizes])
    children = {c: [] for c in bjt.cliques}
    for p, c in bjt.order:
        children[p].append(c)
    wide = sorted(bjt.cliques, key=lambda c: -len(children[c]))[:5]
    rng = np.random.default_rng(0)
    for c in wide:
        t, ls = bjt.pot[c]
        ops = [(t, ls)]
        for k in children[c]:
            sep = [v for v in ls if v in k]
            ops.append((E.to_device(rng.random([bjt.card[v] for v in sep] + [n])), sep + [E.ROW]))
        print("clique", len(ls), "vars, size", bjt.sizes[c], "children", len(children[c]),
              "sep sizes", [o[0].shape for o in ops[1:]][:10])
        for cut in (2, 4, 8):
            sub = ops[:cut]
            out = E.product_n(sub, ls + [E.ROW])
            timer = HipTimer()
            timer.start()
            for _ in range(5):
                E.product_n(sub, ls + [E.ROW], out=out)
            us = timer.stop_ms() * 1e3 / 5
            print(f"  {cut} ops: {us:.1f} us  write {out.numel() * 8 / us / 1e3:.0f} GB/s  out {tuple(out.shape)} "
                  f"strides {[tuple(o.stride()) for o, _ in sub]}")


if __name__ == "__main__":
    main()
