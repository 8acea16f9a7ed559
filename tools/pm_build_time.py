#!/usr/bin/env python3
"""Schedule build time of the C4 batched-BP program (specialised kernel compiles included) and the
number of specialised product+marginal kernels it binds.  python tools/pm_build_time.py [rows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    import torch

    t0 = time.perf_counter()
    sch = bjt.schedule(n, leaves, graph=False, marginals=False)
    t1 = time.perf_counter()
    sch.prog.run()  # lowers, merges per level, compiles the launched kernels (parallel), runs once
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rows {n}: schedule record {t1 - t0:.2f} s, first run (merge + compile) {t2 - t1:.2f} s, "
          f"specialised handles {len(sch.prog._pm_bound)}, launches {len(sch.prog)}, "
          f"PGM_PM_JIT_MIN={os.environ.get('PGM_PM_JIT_MIN', 'default')}")


if __name__ == "__main__":
    main()
