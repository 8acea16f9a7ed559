#!/usr/bin/env python3
"""Per-step HBM-side traffic of the C4 schedule (pathfinder, 4,000 rows) from rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c4pmc_fetch -o f -- python3 tools/c4_step_pmc.py run OUT.json
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c4pmc_write -o w -- python3 tools/c4_step_pmc.py run OUT.json
    python3 tools/c4_step_pmc.py summarize OUT.json gpurun_out/c4pmc_fetch gpurun_out/c4pmc_write

run: builds the levelled schedule without a graph, replays its steps once to warm up and once more; writes
the steps' notes and algorithmic bytes.  summarize: the last len(steps) dispatches of each pass are the
steps in order; FETCH_SIZE doubled (gfx950 counts wide streaming reads at half, MI355X guide) and WRITE_SIZE
(KB) against each step's algorithmic bytes."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out):
    import torch

    from pgmpy_amd import _native as N
    from pgmpy_amd.inference.bp_batch import BatchedJunctionTree
    from pgmpy_amd.inference.EliminationOrder import junction_tree_from_model
    from pgmpy_amd.utils import get_example_model

    rows = int(os.environ.get("ROWS", "4000"))
    m = get_example_model("pathfinder")
    bjt = BatchedJunctionTree(junction_tree_from_model(m))
    leaves = sorted(v for v in m.nodes() if m.out_degree(v) == 0)
    sch = bjt.schedule(rows, leaves, graph=False, marginals=False)
    prog = sch.prog
    prog.run()
    torch.cuda.synchronize()
    prog.run()
    torch.cuda.synchronize()
    json.dump({"rows": rows, "notes": prog.notes, "bytes": prog.step_bytes, "levels": prog.step_levels,
               "floor_bytes_per_calibration": bjt.bytes_per_calibration()}, open(out, "w"))


def counters(d, name):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == name]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows]


def summarize(meta, dfetch, dwrite):
    m = json.load(open(meta))
    n = len(m["notes"])
    fetch = counters(dfetch, "FETCH_SIZE")[-n:]
    write = counters(dwrite, "WRITE_SIZE")[-n:]
    tot_f = 2 * sum(fetch) * 1024
    tot_w = sum(write) * 1024
    alg = sum(m["bytes"])
    out = {"rows": m["rows"], "steps": n, "fetch_bytes_x2": tot_f, "write_bytes": tot_w,
           "hbm_side_bytes": tot_f + tot_w, "step_algorithmic_bytes": alg,
           "floor_bytes": m["floor_bytes_per_calibration"] * m["rows"],
           "ratio_to_step_bytes": (tot_f + tot_w) / alg,
           "ratio_to_floor": (tot_f + tot_w) / (m["floor_bytes_per_calibration"] * m["rows"]), "top": []}
    order = sorted(range(n), key=lambda i: -(2 * fetch[i] + write[i]))
    for i in order[:12]:
        out["top"].append({"step": i, "level": m["levels"][i] if i < len(m["levels"]) else None,
                           "fetch_MB_x2": 2 * fetch[i] * 1024 / 1e6, "write_MB": write[i] * 1024 / 1e6,
                           "alg_MB": m["bytes"][i] / 1e6, "note": m["notes"][i][:110]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summarize(sys.argv[2], sys.argv[3], sys.argv[4])
