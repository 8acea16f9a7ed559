#!/usr/bin/env python3
"""The timed dispatches of a bench.py C3 run in a rocprofv3 kernel trace: the dispatches of `kernel`
in start-time order, [first, first + K) = the timed window (first = warmup + one acquire dispatch per
queue), their GPU span (earliest start to latest end) / K — the figure bench.py's roofline.kernel_ms
reports from the queues' own timestamps — and their mean own duration.  Prints one JSON line.

    python tools/trace_span.py <kernel_trace.csv> <bench.json> [kernel]"""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else None
    b = json.load(open(bench))
    rl = b["roofline"]
    kernel = kernel or rl["kernel"]
    K = int(b["steps"])
    cfg = b["config"]
    first = max(int(b["warmup"]), int(cfg.get("batches", 1))) + (int(cfg.get("queues", 1)) if cfg.get(
        "acquire_before_window") else 0)
    rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].split("(")[0].strip() == kernel]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    win = rows[first:first + K]
    s0 = min(int(r["Start_Timestamp"]) for r in win)
    s1 = max(int(r["End_Timestamp"]) for r in win)
    own = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win]
    span_ms = (s1 - s0) / 1e6 / K
    bpl = rl["bytes_per_launch"] if "bytes_per_step" not in rl else rl["bytes_per_step"]
    out = {"kernel": kernel, "dispatches_in_trace": len(rows), "window": [first, first + K],
           "trace_span_ms_per_step": span_ms, "trace_mean_dispatch_ms": sum(own) / len(own) / 1e6,
           "bench_kernel_ms": rl["kernel_ms"], "ratio_trace_over_bench": span_ms / rl["kernel_ms"],
           "trace_frac": bpl / (span_ms * 1e-3) / 1e9 / rl["peak"], "bench_frac": rl["frac"],
           "bench_frac_wall": rl.get("frac_wall"), "bench_value": b["value"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
