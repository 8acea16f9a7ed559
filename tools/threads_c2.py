#!/usr/bin/env python3
"""Aggregate C2 query throughput from 1 and 8 threads sharing one VariableElimination (munin, the
reference's 20 rows)."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "munin_c2_rows.json")))
    q = g["variables"]
    rows = [r["evidence"] for r in g["rows"]]
    ve = VariableElimination(get_example_model("munin"))
    for r in rows:
        ve.query(q, r, show_progress=False)
    torch.cuda.synchronize()
    out = {}
    for nt in (1, 8):
        per = 400

        def work(k0):
            for k in range(per):
                ve.query(q, rows[(k0 + k) % 20], show_progress=False)

        ths = [threading.Thread(target=work, args=(i,)) for i in range(nt)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        out[nt] = nt * per / dt
    print(json.dumps({"direct": os.environ.get("PGM_QUERY_DIRECT", "1"), "queries_per_s": out}))


if __name__ == "__main__":
    main()
