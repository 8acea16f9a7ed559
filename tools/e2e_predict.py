#!/usr/bin/env python3
"""End-to-end predict / predict_probability on a DataFrame (host data in, DataFrame out) on the munin
C3 template, for an object frame of state names and a pandas Categorical frame (f-4 evidence
ingestion).  Checks the categorical results equal the object results.  Prints one JSON line.
python tools/e2e_predict.py [rows]"""
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import pandas as pd
    import torch

    from pgmpy_amd.inference import batch as B
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import codes_to_frame, forward_sample_codes

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, n, seed=42)
    keep = [v for v in nodes if v not in missing]
    obj = codes_to_frame(m, codes, nodes, columns=keep)
    st = m.states
    pos = {v: i for i, v in enumerate(nodes)}
    cat = pd.DataFrame({c: pd.Categorical.from_codes(codes[pos[c]].astype(np.int8), categories=list(st[c]))
                        for c in keep})
    res = {"rows": n}
    outs = {}
    for fname, df in (("object", obj), ("categorical", cat)):
        for name in ("predict_probability", "predict"):
            fn = getattr(m, name)
            fn(df.iloc[:1000])  # compile the pattern's plan
            torch.cuda.synchronize()
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                out = fn(df)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            outs[(fname, name)] = out
            res[f"{fname}_{name}_rows_per_s"] = n / best
            res[f"{fname}_{name}_s"] = best
        t0 = time.perf_counter()
        ev = B.ingest_frame(m, df)
        torch.cuda.synchronize()
        res[f"{fname}_ingest_s"] = time.perf_counter() - t0
        del ev
    pp_o, pp_c = outs[("object", "predict_probability")], outs[("categorical", "predict_probability")]
    res["categorical_equals_object_probability"] = bool(np.array_equal(pp_o.to_numpy(), pp_c.to_numpy()))
    mo, mc = outs[("object", "predict")], outs[("categorical", "predict")]
    res["categorical_equals_object_map"] = bool((mo[missing].astype(str).to_numpy() == mc[missing].astype(str).to_numpy()).all())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
