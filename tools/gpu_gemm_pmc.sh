# SQ counters of the FP64 GEMM kernel on C2's shapes (one --pmc pass, <= 8 SQ counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -d "$ROOT/gpurun_out/pmc_gemm" -o pmc --output-format csv -- python3 "$ROOT/tools/gemm_bench.py" > "$ROOT/gpurun_out/pmc_gemm.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/pmc_gemm.log"; exit 1; }
python3 - "$ROOT" <<'PY'
import csv, sys, collections
root = sys.argv[1]
import glob
f = glob.glob(root + "/gpurun_out/pmc_gemm/**/pmc_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: round(x) for c, x in v.items()})
PY
