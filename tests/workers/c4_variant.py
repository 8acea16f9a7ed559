"""Worker for tests/test_kernels_gpu.py::test_bp_block_order_knobs_bit_exact: one batched pathfinder
calibration (1,002 rows: block counts that are not multiples of 8) under the environment it is started
with (PGM_PM_XCD / PGM_PM_XPART / PGM_PM_KREV select the block-to-tile order of the specialised steps,
read once per process); saves every clique belief (rows innermost) to OUT.npz.

    python tests/workers/c4_variant.py OUT"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(out):
    import pandas as pd

    from pgmpy_amd.inference.batch import download
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import build_junction_tree
    from pgmpy_amd.utils import get_example_model
    from tests.goldens import load_json

    m = get_example_model("pathfinder")
    meta = load_json("pathfinder_bp.json")
    jt = build_junction_tree(m, [tuple(b) for b in meta["bags"]], [(tuple(a), tuple(b)) for a, b in meta["edges"]])
    base = pd.DataFrame([c["evidence"] for c in meta["cases"]])
    rows = 1002
    cal = BatchedJunctionTree(jt).calibrate_frame(pd.concat([base] * (rows // len(base) + 1),
                                                            ignore_index=True).iloc[:rows])
    np.savez(out, **{f"b{i}": download(t.contiguous()) for i, (t, _) in enumerate(cal.beliefs.values())})


if __name__ == "__main__":
    main(sys.argv[1])
