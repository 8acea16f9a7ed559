"""Worker for tests/test_kernels_gpu.py::test_specialised_kernel_disk_cache (-m gpu).

Builds the batched-BP schedule of pathfinder for 256 forward-sampled rows (its fused
product+marginal steps compile into specialised kernels, cached under $PGM_KERNEL_CACHE), calibrates,
and prints as JSON: the kernels bound, the cache files present afterwards, the schedule build time
and a checksum of every clique belief.
"""
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import codes_to_frame, forward_sample_codes

    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    codes, nodes = forward_sample_codes(m, 256, seed=5)
    df = codes_to_frame(m, codes, nodes, columns=leaves)
    t0 = time.perf_counter()
    sch = bjt.schedule(256, list(df.columns))
    build = time.perf_counter() - t0
    cal = bjt.calibrate_frame(df)
    tot = float(sum(np.asarray(cal.clique_belief(c, r)).sum() for c in bjt.cliques for r in (0, 255)))
    files = sorted(glob.glob(os.path.join(os.environ["PGM_KERNEL_CACHE"], "k*.co")))
    print(json.dumps({"bound": len(sch.prog._pm_bound), "files": len(files), "build_s": build, "checksum": tot}))


if __name__ == "__main__":
    main()
