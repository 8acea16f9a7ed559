#!/usr/bin/env python3
"""Stage times of the public DataFrame API on the munin C3 template (categorical frame, 100k rows):
ingestion (Categorical codes + NaN scan), plan lookup, evidence upload, the fused pass, the output
download and the result frame, each timed alone (median of 5), plus the whole predict_probability /
predict calls.  Prints one JSON line.  python tools/e2e_profile.py [rows]"""
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(fn, reps=5):
    import torch

    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3, r


def main():
    import pandas as pd

    from pgmpy_amd.inference import batch as B
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, n, seed=42)
    keep = [v for v in nodes if v not in missing]
    st = m.states
    pos = {v: i for i, v in enumerate(nodes)}
    cat = pd.DataFrame({c: pd.Categorical.from_codes(codes[pos[c]].astype(np.int8), categories=list(st[c]))
                        for c in keep})
    cols = list(cat.columns)
    col_of = {c: i for i, c in enumerate(cols)}
    order = list(set(m.nodes()) - set(cols))
    res = {"rows": n}
    m.predict_probability(cat.iloc[:1000])
    m.predict(cat.iloc[:1000])
    res["predict_probability_ms"], pp_fast = med(lambda: m.predict_probability(cat))
    res["predict_ms"], p_fast = med(lambda: m.predict(cat))
    os.environ["PGM_API_APPEND"] = "concat"
    res["predict_concat_ms"], _ = med(lambda: m.predict(cat))
    os.environ.pop("PGM_API_APPEND")
    B.FAST_MIN_ROWS = 10 ** 12  # the per-pattern path (r03) for comparison
    res["predict_probability_grouped_ms"], pp_slow = med(lambda: m.predict_probability(cat))
    res["predict_grouped_ms"], p_slow = med(lambda: m.predict(cat))
    B.FAST_MIN_ROWS = 50_000
    res["fast_equals_grouped_probability"] = bool(pp_fast.equals(pp_slow))
    res["fast_equals_grouped_predict"] = bool((p_fast[order].astype(str).to_numpy() == p_slow[order].astype(str).to_numpy()).all()
                                              and list(p_fast.columns) == list(p_slow.columns))
    res["rows_per_s"] = {"predict_probability": n / res["predict_probability_ms"] * 1e3,
                         "predict": n / res["predict_ms"] * 1e3}
    res["ingest_columnar_ms"], ev = med(lambda: B.ingest_columnar(m, cat, cols))
    ptrs = [a.__array_interface__["data"][0] for a in ev.raws]
    import ctypes

    from pgmpy_amd import _native as N

    arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
    flag = np.zeros(len(ptrs), dtype=np.uint8)
    for t in (1, 4, 16):
        res[f"nan_scan_{t}t_ms"], _ = med(lambda: N.lib().pgm_host_any_negative_i8(
            arr, len(ptrs), n, flag.ctypes.data_as(ctypes.c_void_p), t))
    mask, rows = ev.groups[0]
    res["groups"] = len(ev.groups)
    observed = [cols[j] for j in range(len(cols)) if mask[j]]
    res["get_plan_ms"], plan = med(lambda: B.get_plan(m, order, observed, col_of))
    used = [col_of[v] for v in plan.ev_used]
    res["host_codes_ms"], hc = med(lambda: ev.host_codes_for(used, rows))
    res["upload_ms"], d = med(lambda: B.upload_codes(hc))
    cp = plan.compact()
    out = cp.alloc_outputs(n, marginals=True)
    res["run_ms"], _ = med(lambda: cp.run(d, n, 0, n, out))
    res["download_ms"], host = med(lambda: B.download(out["marg"]))
    names = [v + "_" + str(s) for v in order for s in m.get_cpds(v).state_names[v]]
    res["frame_from_block_ms"], _ = med(lambda: pd.DataFrame(host.T, columns=names, index=cat.index))
    # the direct path's own stages, timed alone on the same frame
    ing = B._ingest(m, cat)
    res["direct_ingest_ms"], ing = med(lambda: B._ingest(m, cat))
    res["direct_plan_ms"], plan = med(lambda: B._single_fused_plan(m, cat, *ing, order))
    res["direct_fused_to_host_ms"], marg = med(lambda: B._fused_to_host(plan, ing[2], ing[0], ing[1], n, True))
    res["direct_frame_ms"], _ = med(lambda: pd.DataFrame(marg.T, columns=names, index=cat.index, copy=False))
    res["direct_nodes_minus_columns_ms"], _ = med(lambda: list(set(m.nodes()) - set(cat.columns)))
    import cProfile
    import io
    import pstats

    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        m.predict_probability(cat)
    pr.disable()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(14)
    res["cprofile_predict_probability_x5"] = buf.getvalue().splitlines()[-22:]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
