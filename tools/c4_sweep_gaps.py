#!/usr/bin/env python3
"""C4's sweep inside the timed loop, from a rocprofv3 kernel trace of `bench.py --workload c4`: per launch
position of the sweep, the median kernel duration and the median gap from the previous kernel's end to its
start, over the sweeps of the trace (the sweep's period is found from the kernel-name sequence).  Says how
much of a sweep is kernels and how much is the boundaries between them.

    python3 tools/c4_sweep_gaps.py TRACE_kernel_trace.csv [period]"""
import csv
import gzip
import json
import statistics
import sys


def main(trace, period=None):
    with (gzip.open(trace, "rt") if trace.endswith(".gz") else open(trace)) as fh:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48], r["Queue_Id"])
                for r in csv.DictReader(fh)]
    rows.sort()
    # the sweep's launches (specialised steps, level batches, generic product kernels), not the copies and
    # contractions of the parity readout that follows the timed loop
    first_sweep = [i for i, r in enumerate(rows) if r[2].startswith(("pgm_pm", "k_batch", "k_productn"))]
    rows = [rows[i] for i in first_sweep]
    names = [r[2] for r in rows]
    if period is None:  # the smallest period whose name sequence repeats over the first 300 launches
        tail = names[:300]
        period = next(p for p in range(2, 100) if sum(tail[i] == tail[i + p] for i in range(len(tail) - p))
                      >= 0.95 * (len(tail) - p))
    period = int(period)
    # align on the sweep's first launch: the position whose gap before it is largest on average
    n = (len(rows) // period) * period
    rows = rows[:n]
    gaps_all = [0.0] + [(rows[i][0] - rows[i - 1][1]) / 1e3 for i in range(1, len(rows))]
    shift = max(range(period), key=lambda s: statistics.median(gaps_all[s::period][1:]))
    rows = rows[shift:]
    sweeps = [rows[i:i + period] for i in range(0, len(rows) - period + 1, period)]
    sweeps = sweeps[1:]  # the first is a cold warm-up
    out = {"trace": trace, "period": period, "sweeps": len(sweeps), "positions": []}
    kern_tot = gap_tot = 0.0
    for p in range(period):
        d = statistics.median((s[p][1] - s[p][0]) / 1e3 for s in sweeps)
        g = statistics.median((s[p][0] - s[p - 1][1]) / 1e3 for s in sweeps) if p else None
        kern_tot += d
        gap_tot += g or 0.0
        out["positions"].append({"p": p, "kernel": sweeps[0][p][2], "us": round(d, 1),
                                 "gap_before_us": None if g is None else round(g, 2)})
    span = statistics.median((s[-1][1] - s[0][0]) / 1e3 for s in sweeps)
    out.update({"kernel_sum_us": round(kern_tot, 1), "gap_sum_us": round(gap_tot, 1), "sweep_span_us": round(span, 1)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
