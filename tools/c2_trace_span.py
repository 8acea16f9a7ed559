#!/usr/bin/env python3
"""C2's queries in a rocprofv3 kernel trace of `bench.py --workload c2`.

    python tools/c2_trace_span.py TRACE_kernel_trace.csv BENCH_LINE.json [launches_per_query]

The queries run as AQL chains on the query queue (Queue_Id of the pgm_pm dispatches).  The last
(warmup + steps + 20 parity + 20 mass) chains of that queue are taken as the run's queries in issue
order; the timed window is the `steps` chains after the cold query and the warmup.  For each timed chain:
its GPU span (first kernel start -> last kernel end) and the sum of its kernels' durations; the gaps
between consecutive timed chains are the host's part of a query (Python, codes, doorbell, the wait).
Reports the medians and the window's time per query recomputed from the trace (chain start to chain
start) against the line's own value (profiled run)."""
import csv
import json
import statistics
import sys


def main(trace, line_path, per_query=None):
    with open(line_path) as fh:
        line = json.loads(fh.read().strip().splitlines()[-1])
    per_query = int(per_query or line.get("launches_per_query") or 20)
    rows = []
    import gzip

    with (gzip.open(trace, "rt") if trace.endswith(".gz") else open(trace)) as fh:
        for r in csv.DictReader(fh):
            if r["Kernel_Name"].startswith("pgm_pm"):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]))
    queues = {}
    for a, b, q in rows:
        queues.setdefault(q, []).append((a, b))
    q, ks = max(queues.items(), key=lambda kv: len(kv[1]))  # the query queue carries the chains
    ks.sort()
    n_chains = len(ks) // per_query
    assert len(ks) % per_query == 0, (len(ks), per_query)
    chains = [ks[i * per_query:(i + 1) * per_query] for i in range(n_chains)]
    steps, warm = int(line["steps"]), int(line["warmup"])
    # issue order: cold query, warmup, steps, then the parity pass (20 queries + 20 unnormalised reads)
    timed = chains[1 + warm:1 + warm + steps]
    spans = [(c[-1][1] - c[0][0]) / 1e3 for c in timed]
    busy = [sum(b - a for a, b in c) / 1e3 for c in timed]
    gaps = [(timed[i + 1][0][0] - timed[i][-1][1]) / 1e3 for i in range(len(timed) - 1)]
    start_to_start_us = (timed[-1][0][0] - timed[0][0][0]) / 1e3  # len - 1 whole queries
    out = {
        "trace": trace, "queue": q, "chains_in_trace": n_chains, "launches_per_query": per_query,
        "timed_chains": len(timed),
        "gpu_span_us": {"median": statistics.median(spans), "min": min(spans), "max": max(spans)},
        "kernel_sum_us": {"median": statistics.median(busy)},
        "host_gap_us": {"median": statistics.median(gaps)} if gaps else None,
        "trace_us_per_query": start_to_start_us / (len(timed) - 1) if len(timed) > 1 else None,
        "line_us_per_query_profiled": line["value"] * 1e6,
    }
    out["trace_over_line"] = out["trace_us_per_query"] / out["line_us_per_query_profiled"]
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
