# (specialised + merged kernels) per-dispatch FETCH_SIZE / WRITE_SIZE of the C4 schedule's kernels (4000 rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $ROOT/gpurun_out/pmc2_c4_$C -o pmc --output-format csv -- python3 $ROOT/bench.py --workload c4 --rows 4000 --steps 1 --warmup 1 > /dev/null 2> $ROOT/gpurun_out/pmc2_c4_$C.err || { tail -20 $ROOT/gpurun_out/pmc2_c4_$C.err; exit 1; }
done
cd $ROOT && python3 - <<'PY'
import csv, collections
rows = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for r in csv.DictReader(open(f"gpurun_out/pmc2_c4_{c}/pmc_counter_collection.csv")):
        key = (r["Dispatch_Id"], r["Kernel_Name"][:60])
        rows.setdefault(key, {})[c] = float(r["Counter_Value"])
tr = {}
for r in csv.DictReader(open("gpurun_out/pmc2_c4_FETCH_SIZE/pmc_kernel_trace.csv")):
    tr[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
items = sorted(rows.items(), key=lambda kv: -(kv[1].get("FETCH_SIZE", 0) + kv[1].get("WRITE_SIZE", 0)))
tot = collections.Counter()
for (did, name), v in items:
    tot["FETCH_KB"] += v.get("FETCH_SIZE", 0); tot["WRITE_KB"] += v.get("WRITE_SIZE", 0)
print("totals (both steps) KB", dict(tot))
for (did, name), v in items[:14]:
    print(did, name[:50], {k: round(x) for k, x in v.items()}, "us", tr.get(did))
PY
