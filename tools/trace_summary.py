#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 kernel_trace.csv: calls, total/median/max us, grid of the slowest."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0][:48]
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    by[name].append((dur, grid))
tot_all = sum(d for v in by.values() for d, _ in v)
print(f"total kernel time {tot_all / 1e3:.2f} ms over {sum(len(v) for v in by.values())} dispatches")
for k, v in sorted(by.items(), key=lambda kv: -sum(d for d, _ in kv[1])):
    v.sort()
    tot = sum(d for d, _ in v)
    print(f"{k:48s} n={len(v):6d} tot={tot / 1e3:8.2f}ms med={v[len(v) // 2][0]:8.1f}us max={v[-1][0]:8.1f}us "
          f"slowest_grid={v[-1][1]}")
