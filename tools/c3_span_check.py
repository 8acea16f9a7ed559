#!/usr/bin/env python3
"""Recompute the C3 line's span-based roofline from its own raw dispatch timestamps.

    python tools/c3_span_check.py profiles/<run>/bench_default.json [...]

The default bench line (bench.py, --launch direct, 4 queues) carries roofline.dispatch_times: every timed
dispatch's HSA start / end ticks and its queue.  From them alone this script recomputes

  * the GPU span per step  = (max end - min start) / freq / steps        (the line's roofline.kernel_ms)
  * achieved               = bytes_per_launch / span per step              (roofline.achieved)
  * frac                   = achieved / peak                               (roofline.frac)

and checks it against the line within 5 %.  It also splits the span the way the ring comparison needs:
per-dispatch durations, how many dispatches are in flight over the span (time-weighted), the ramp
(window start to the first moment four dispatches run) and the tail (last moment four run to the end),
and the steady part's time per step.
"""
import json
import sys


def analyse(line):
    r = line["roofline"]
    dt = r.get("dispatch_times")
    if not dt or not dt.get("dispatches"):
        raise SystemExit("the line carries no roofline.dispatch_times (bench.py before r06, or --launch hip)")
    f = float(dt["freq"])
    ds = sorted(((a, b, q) for q, a, b in dt["dispatches"]), key=lambda x: x[0])
    steps = int(line["steps"])
    assert len(ds) == steps, (len(ds), steps)
    t0 = min(a for a, _, _ in ds)
    t1 = max(b for _, b, _ in ds)
    span_ms = (t1 - t0) / f * 1e3
    per_step_ms = span_ms / steps
    bpl = float(r["bytes_per_launch"])
    achieved = bpl / (per_step_ms * 1e-3) / 1e9
    frac = achieved / float(r["peak"])
    # in-flight count over the span (time-weighted)
    ev = sorted([(a, 1) for a, _, _ in ds] + [(b, -1) for _, b, _ in ds])
    cur, last, busy, weighted, full_first, full_last = 0, t0, 0, 0, None, None
    qn = int(r.get("concurrent_queues") or 1)
    for t, d in ev:
        if cur > 0:
            busy += t - last
            weighted += cur * (t - last)
        if cur >= qn and full_first is None:
            full_first = last
        if cur >= qn:
            full_last = t
        cur += d
        last = t
    durs = [(b - a) / f * 1e3 for a, b, _ in ds]
    out = {
        "steps": steps,
        "span_ms": span_ms,
        "kernel_ms_recomputed": per_step_ms,
        "kernel_ms_line": r["kernel_ms"],
        "achieved_recomputed": achieved,
        "frac_recomputed": frac,
        "frac_line": r["frac"],
        "frac_agrees_within_5pct": abs(frac / r["frac"] - 1) <= 0.05,
        "dispatch_ms": {"mean": sum(durs) / len(durs), "min": min(durs), "max": max(durs)},
        "dispatch_avg_ms_line": r.get("dispatch_avg_ms"),
        "mean_in_flight_over_span": weighted / (t1 - t0),
        "busy_fraction_of_span": busy / (t1 - t0),
        "queues": qn,
    }
    if full_first is not None:
        ramp = (full_first - t0) / f * 1e3
        tail = (t1 - full_last) / f * 1e3
        n_steady = sum(1 for a, b, _ in ds if a >= full_first and b <= full_last)
        out["ramp_ms"] = ramp
        out["tail_ms"] = tail
        out["steady_ms"] = (full_last - full_first) / f * 1e3
        out["steady_dispatches_inside"] = n_steady
    ring = r.get("single_launch_ring") or {}
    if ring.get("ms_per_batch"):
        out["ring_ms_per_batch"] = ring["ms_per_batch"]
        out["span_over_ring"] = per_step_ms / ring["ms_per_batch"]
    return out


def main(paths):
    res = {}
    for p in paths:
        with open(p) as fh:
            line = json.loads(fh.read().strip().splitlines()[-1])
        res[p] = analyse(line)
    print(json.dumps(res, indent=1))
    return 0 if all(v["frac_agrees_within_5pct"] for v in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
