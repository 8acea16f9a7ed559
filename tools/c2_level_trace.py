#!/usr/bin/env python3
"""C2's per-level kernel times and the gaps between them, from a rocprofv3 kernel trace (profiling aid).

    rocprofv3 --kernel-trace -d DIR -o t --output-format csv -- python3 tools/c2_level_trace.py run REPS
    python3 tools/c2_level_trace.py summarize DIR

`run` builds the munin C2 query (bench.py's pattern), then issues REPS complete queries (ve.query: host
work, one graph launch, spin wait) with a 1 ms host pause between them, so each query starts from an idle
GPU as in the bench.  `summarize` takes the last REPS groups of launches from the trace (one group per
query: launches closer than 50 us to the previous one) and reports per position in the group the median
kernel duration and the median gap from the previous kernel's end to this one's start."""
import csv
import glob
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(reps):
    import random

    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("munin")
    leaves = sorted(n for n in m.nodes() if m.out_degree(n) == 0)
    roots = sorted(n for n in m.nodes() if m.in_degree(n) == 0)
    rng = random.Random(100000)
    ev_vars = rng.sample(leaves, 100)
    q = [rng.choice(roots)]
    codes, nodes = forward_sample_codes(m, 1, seed=0)
    evidence = {v: m.states[v][codes[nodes.index(v), 0]] for v in ev_vars}
    ve = VariableElimination(m)
    for _ in range(20):
        ve.query(q, evidence, show_progress=False)
    torch.cuda.synchronize()
    lat = []
    for _ in range(reps):
        time.sleep(1e-3)
        t0 = time.perf_counter()
        ve.query(q, evidence, show_progress=False)
        lat.append(time.perf_counter() - t0)
    print(f"queries: {reps}, median host-measured latency {statistics.median(lat) * 1e3:.4f} ms")


def summarize(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and s - cur[-1][1] > 50_000:
            groups.append(cur)
            cur = []
        cur.append((s, e, r["Kernel_Name"].split("(")[0][:48]))
    if cur:
        groups.append(cur)
    n = statistics.mode(len(g) for g in groups)
    groups = [g for g in groups if len(g) == n][-100:]
    print(f"{len(groups)} queries of {n} launches each")
    tot_k = tot_g = 0.0
    for i in range(n):
        dur = statistics.median((g[i][1] - g[i][0]) / 1e3 for g in groups)
        gap = statistics.median((g[i][0] - g[i - 1][1]) / 1e3 for g in groups) if i else 0.0
        tot_k += dur
        tot_g += gap
        print(f"{i:3d} {dur:7.2f} us  gap {gap:6.2f} us  {groups[0][i][2]}")
    span = statistics.median((g[-1][1] - g[0][0]) / 1e3 for g in groups)
    print(f"kernels {tot_k:.1f} us + gaps {tot_g:.1f} us; first start to last end {span:.1f} us (medians)")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 200)
    else:
        summarize(sys.argv[2])
