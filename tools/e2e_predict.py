#!/usr/bin/env python3
"""End-to-end predict / predict_probability on a DataFrame (host data in, DataFrame out):
phase breakdown on the munin C3 template.  python tools/e2e_predict.py [rows]"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import batch as B
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import codes_to_frame, forward_sample_codes

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    m = get_example_model("munin")
    missing = random.Random(0).sample(sorted(m.nodes()), 3)
    codes, nodes = forward_sample_codes(m, n, seed=42)
    df = codes_to_frame(m, codes, nodes).drop(columns=missing)
    for name, fn in (("predict_probability", m.predict_probability), ("predict", m.predict)):
        fn(df.iloc[:1000])  # compile the pattern's plan
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn(df)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{name}: {n} rows in {dt:.3f} s = {n / dt:,.0f} rows/s (DataFrame in -> DataFrame out), out {out.shape}")
    t0 = time.perf_counter()
    enc = B.encode_frame(m, df)
    t1 = time.perf_counter()
    d = B.upload_codes(enc)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"  encode_frame {t1 - t0:.3f} s, upload {enc.nbytes / 1e6:.0f} MB {t2 - t1:.3f} s")


if __name__ == "__main__":
    main()
