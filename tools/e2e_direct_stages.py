#!/usr/bin/env python3
"""The public API's direct path (inference.batch._direct_categorical) for the bench's api_e2e frame (munin,
100 k rows, 1,038 Categorical evidence columns, 3 missing): the whole predict_probability call and its
parts timed separately (medians over N calls): the direct path alone, the native NaN scan of every column
alone, the Python walk of the columns alone, the result DataFrame built on the pinned block, and a
13.6 MB pinned D2H copy alone.

    python3 tools/e2e_direct_stages.py [N]"""
import ctypes
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n_calls=30):
    n_calls = int(n_calls)
    import numpy as np
    import pandas as pd
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference import batch as B
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    model = get_example_model("munin")
    missing = set(random.Random(0).sample(sorted(model.nodes()), 3))
    codes_all, nodes = forward_sample_codes(model, 100_000, seed=42)
    st = model.states
    pos = {v: i for i, v in enumerate(nodes)}
    keep = [v for v in nodes if v not in missing]
    df = pd.DataFrame({c: pd.Categorical.from_codes(codes_all[pos[c]].astype(np.int8), categories=list(st[c]))
                       for c in keep})
    model.predict_probability(df.iloc[:1000])
    for _ in range(3):
        model.predict_probability(df)
    torch.cuda.synchronize()

    def med(fn):
        ts = []
        for _ in range(n_calls):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e6

    order = sorted(missing, key=lambda v: list(model.nodes()).index(v))
    order = [v for v in model.nodes() if v in missing]
    out = {"rows": len(df), "columns": len(keep), "host_threads": B._host_threads()}
    out["whole_us"] = med(lambda: model.predict_probability(df))
    d = B._direct_categorical(model, df, order, True)
    out["direct_path_taken"] = d is not None
    out["direct_us"] = med(lambda: B._direct_categorical(model, df, order, True))
    arrays = df._mgr.arrays
    L = N.lib()
    ptrs = (ctypes.c_void_p * len(arrays))(*[a._codes.ctypes.data for a in arrays])
    flags = np.zeros(len(arrays), dtype=np.uint8)
    out["scan_all_columns_us"] = med(lambda: N.check(L.pgm_host_any_negative_i8(
        ptrs, len(arrays), len(df), flags.ctypes.data_as(ctypes.c_void_p), B._host_threads())))

    def walk():
        cat_t = B.pd_categorical()
        i8 = np.dtype(np.int8)
        for c0 in range(0, len(arrays), B._SCAN_CHUNK):
            part = arrays[c0:c0 + B._SCAN_CHUNK]
            assert all(type(a) is cat_t for a in part)
            raws = [a._codes for a in part]
            assert all(r.dtype is i8 and r.flags.c_contiguous for r in raws)
            [a.dtype for a in part]
            (ctypes.c_void_p * len(raws))(*[ctypes.addressof(ctypes.c_char.from_buffer(r)) for r in raws])

    out["walk_us"] = med(walk)
    if d is not None:
        marg = d[1]
        names = B._result_columns(model, order)
        out["result_frame_us"] = med(lambda: pd.DataFrame(marg.T, columns=names, index=df.index, copy=False))
        dev = torch.empty(marg.shape, dtype=torch.float64, device="cuda")
        s = N.stream_handle()
        out["d2h_%d_MB_us" % (marg.nbytes >> 20)] = med(lambda: N.check(L.pgm_memcpy_d2h_async(
            marg.ctypes.data_as(ctypes.c_void_p), N.ptr(dev), marg.nbytes, s)))
    print(json.dumps(out, indent=1))
    import cProfile
    import io
    import pstats

    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        B._direct_categorical(model, df, order, True)
    pr.disable()
    sio = io.StringIO()
    pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(25)
    print(sio.getvalue())


if __name__ == "__main__":
    main(*sys.argv[1:])
