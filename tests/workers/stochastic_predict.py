"""Worker for tests/test_inference_gpu.py::test_predict_stochastic_matches_reference (-m gpu).

Run with PYTHONHASHSEED=0 (the hash seed the fixture was generated under): the reference's factor
over {missing variables} U {row's NaN columns} is ordered by set iteration, which this process then
reproduces.  Runs predict(stochastic=True, seed) on the fixture's case through the HIP path and
prints the number of cells that differ from the reference's output as JSON.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(case):
    import pandas as pd

    from pgmpy_amd.utils import get_example_model

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "alarm_predict_stochastic.json")))
    c = g[case]
    m = get_example_model("alarm")
    data = pd.DataFrame(c["rows"], columns=c["columns"]).astype(object)
    data = data.where(pd.notna(data), np.nan)
    pred = m.predict(data, stochastic=True, seed=g["seed"])
    got = pred[c["predict_columns"]].astype(str).to_numpy()
    exp = pd.DataFrame(c["predict"], columns=c["predict_columns"]).astype(str).to_numpy()
    print(json.dumps({"cells": int(got.size), "mismatch": int((got != exp).sum()),
                      "columns_equal": list(pred.columns) == c["predict_columns"]}))


if __name__ == "__main__":
    main(sys.argv[1])
