#!/usr/bin/env python3
"""C5's rotating roofline (bench.py --workload c5: roofline.kernel_ms over `launches` back-to-back
launches rotating over HBM-sized buffers) against a rocprofv3 kernel trace of the same command: the
last `launches` dispatches of the roofline's kernel are those launches (nothing launches it after
them).  Reports their mean own duration and their span / launches beside the bench's HIP-event figure.

    python tools/c5_trace_check.py <kernel_trace.csv> <bench.json>"""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    rl = b["roofline"]
    n = int(rl["launches"])
    rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].split("(")[0].strip() == rl["kernel"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    win = rows[-n:]
    own = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win]
    span = (max(int(r["End_Timestamp"]) for r in win) - min(int(r["Start_Timestamp"]) for r in win)) / 1e6 / n
    mean = sum(own) / len(own) / 1e6
    out = {"kernel": rl["kernel"], "dispatches_in_trace": len(rows), "launches": n,
           "trace_mean_dispatch_ms": mean, "trace_span_ms_per_launch": span, "bench_kernel_ms": rl["kernel_ms"],
           "ratio_trace_mean_over_bench": mean / rl["kernel_ms"], "ratio_trace_span_over_bench": span / rl["kernel_ms"],
           "trace_frac_mean": rl["bytes_per_launch"] / (mean * 1e-3) / 1e9 / rl["peak"], "bench_frac": rl["frac"],
           "working_set_over_mall": rl.get("working_set_over_mall")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
