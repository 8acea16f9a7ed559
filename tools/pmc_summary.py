#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run (gpurun_out/prof_TAG, pmc_fetch_TAG, pmc_write_TAG) into
profiles/TAG_kernel_stats.csv and profiles/TAG_pmc_pgm_rows_jit.json (+ profiles/pmc_pgm_rows_jit.json,
which bench.py reads for roofline.traffic).  python tools/pmc_summary.py TAG [KERNEL]
(KERNEL: pgm_rows_jit, default, or pgm_rows_jit2 — the kernel the bench's bound launch runs)"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "pgm_rows_jit"


def is_kernel(name):
    """name is KERNEL (possibly with a suffix such as ".kd"), not a longer kernel name"""
    return name.startswith(KERNEL) and not name[len(KERNEL):len(KERNEL) + 1].isalnum()


def counter(tag, what, name):
    vals = []
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{what}_{tag}", "**", "*counter_collection.csv"),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            if is_kernel(r["Kernel_Name"]) and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return vals


def main(tag):
    stats = glob.glob(os.path.join(ROOT, "gpurun_out", f"prof_{tag}", "**", "*kernel_stats.csv"), recursive=True)
    avg = None
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            if is_kernel(r["Name"]):
                avg = float(r["AverageNs"])
    fetch, write = counter(tag, "fetch", "FETCH_SIZE"), counter(tag, "write", "WRITE_SIZE")
    f_kb, w_kb = sum(fetch) / len(fetch), sum(write) / len(write)
    out = {"tag": tag, "kernel": KERNEL, "rows_per_launch": 100000, "launches_profiled": len(fetch),
           "FETCH_SIZE_KB": f_kb, "WRITE_SIZE_KB": w_kb, "fetch_correction": 1,
           "hbm_bytes_per_launch": (f_kb + w_kb) * 1024, "rocprof_avg_ns": avg}
    for p in (f"{tag}_pmc_{KERNEL}.json", f"pmc_{KERNEL}.json"):
        with open(os.path.join(ROOT, "profiles", p), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
