#!/usr/bin/env python3
"""Per-step kernel durations of the C4 schedule from rocprofv3 kernel traces of `c4_step_pmc.py run`
(the last len(steps) dispatches are the steps in order), side by side for several runs (e.g. an A/B knob).

    python3 tools/c4_step_times.py META.json LABEL=TRACE_DIR [LABEL=TRACE_DIR ...]"""
import csv
import glob
import json
import os
import sys


def durations(d, n):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows], \
        [r["Kernel_Name"].split("(")[0][:40] for r in rows]


def main():
    m = json.load(open(sys.argv[1]))
    n = len(m["notes"])
    runs = [a.split("=", 1) for a in sys.argv[2:]]
    cols = {lab: durations(d, n) for lab, d in runs}
    labs = [lab for lab, _ in runs]
    out = {"steps": n, "total_us": {lab: sum(cols[lab][0]) for lab in labs}, "per_step": []}
    for i in range(n):
        out["per_step"].append({"i": i, "level": m["levels"][i] if i < len(m["levels"]) else None,
                                "note": m["notes"][i][:90], "MB": m["bytes"][i] / 1e6 if i < len(m["bytes"]) else None,
                                **{lab: round(cols[lab][0][i], 1) for lab in labs}})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
