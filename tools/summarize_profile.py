#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run into profiles/ (committed evidence).

  python tools/summarize_profile.py TAG KERNEL ROWS_PER_LAUNCH

Writes profiles/<TAG>_kernel_stats.csv (rocprofv3 --kernel-trace --stats) and
profiles/pmc_<KERNEL>.json: per-launch FETCH_SIZE / WRITE_SIZE (KB, separate
--pmc passes) and hbm_bytes_per_launch = (FETCH_SIZE + WRITE_SIZE) * 1024.
gfx950 note (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads 1/2 of the bytes of a
WIDE (16 B/lane) coalesced stream; the row kernels read 1-byte codes per lane, and their
FETCH_SIZE matches the algorithmic code bytes without that correction, so no
doubling is applied (recorded as "fetch_correction": 1).
"""
import csv
import json
import os
import shutil
import statistics
import sys

tag, kernel, rows = sys.argv[1], sys.argv[2], int(sys.argv[3])
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_dir = os.path.join(root, "gpurun_out")
prof = os.path.join(root, "profiles")
os.makedirs(prof, exist_ok=True)
shutil.copy(os.path.join(out_dir, f"prof_{tag}", "trace_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))


def counter(path, name):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Kernel_Name"].split("<")[0].split("(")[0].endswith(kernel) and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return vals


fetch = counter(os.path.join(out_dir, f"pmc_fetch_{tag}", "pmc_counter_collection.csv"), "FETCH_SIZE")
write = counter(os.path.join(out_dir, f"pmc_write_{tag}", "pmc_counter_collection.csv"), "WRITE_SIZE")
durs = []
with open(os.path.join(out_dir, f"prof_{tag}", "trace_kernel_stats.csv")) as f:
    for r in csv.DictReader(f):
        if r["Name"].split("<")[0].split("(")[0].endswith(kernel):
            avg_ns = float(r["AverageNs"])
fetch_kb, write_kb = statistics.median(fetch), statistics.median(write)
summary = {
    "tag": tag, "kernel": kernel, "rows_per_launch": rows, "launches_profiled": len(fetch),
    "FETCH_SIZE_KB": fetch_kb, "WRITE_SIZE_KB": write_kb, "fetch_correction": 1,
    "hbm_bytes_per_launch": (fetch_kb + write_kb) * 1024.0,
    "rocprof_avg_ns": avg_ns,
}
with open(os.path.join(prof, f"pmc_{kernel}.json"), "w") as f:
    json.dump(summary, f, indent=1)
shutil.copy(os.path.join(prof, f"pmc_{kernel}.json"), os.path.join(prof, f"{tag}_pmc_{kernel}.json"))
print(json.dumps(summary))
