#!/usr/bin/env python3
"""Where a single query's GPU time goes (C2 / C1), from a rocprofv3 kernel trace of `bench.py --workload c2`:
dispatches sorted by start time are split into queries at host gaps longer than `gap_us` (the host work
between two queries); for the last `n` queries it reports dispatches per query, the GPU span (first start to
last end), the summed kernel durations, the summed gaps between consecutive dispatches, and the mean
duration per kernel name.  Prints one JSON object.

    python tools/c2_trace.py <kernel_trace.csv> [n=20] [gap_us=25]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    trace = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    gap_us = float(sys.argv[3]) if len(sys.argv) > 3 else 25.0
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > gap_us * 1e3:
            groups.append(cur)
            cur = []
        cur.append((s, e, r["Kernel_Name"].split("(")[0].strip()))
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        groups.append(cur)
    tail = groups[-n:]
    sizes = sorted({len(g) for g in tail})
    spans, busy, gaps = [], [], []
    per_kernel = defaultdict(list)
    for g in tail:
        spans.append((g[-1][1] - g[0][0]) / 1e3)
        busy.append(sum(e - s for s, e, _ in g) / 1e3)
        gaps.append(sum(max(0, g[i + 1][0] - g[i][1]) for i in range(len(g) - 1)) / 1e3)
        for s, e, k in g:
            per_kernel[k].append((e - s) / 1e3)
    mean = lambda xs: sum(xs) / len(xs)
    print(json.dumps({
        "queries": len(tail), "dispatches_per_query": sizes,
        "span_us": mean(spans), "kernel_busy_us": mean(busy), "gaps_us": mean(gaps),
        "per_kernel_us": {k: {"n_per_query": len(v) / len(tail), "mean_us": mean(v)}
                          for k, v in sorted(per_kernel.items(), key=lambda kv: -sum(kv[1]))},
    }, indent=1))


if __name__ == "__main__":
    main()
