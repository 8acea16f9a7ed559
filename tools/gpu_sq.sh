# SQ counters for the fused row kernel: one variant, one batch size, two PMC passes.
#   bash tools/gpu_sq.sh TAG ROWS VARIANT
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"; TAG=${1:-sq}; ROWS=${2:-1000000}; VAR=${3:-lds_values}
cd /tmp && export TMPDIR=/tmp
pass() {
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$ROOT/gpurun_out/$TAG" -o pmc --output-format csv -- \
    python3 "$ROOT/tools/rows_sweep.py" --rows $ROWS --reps 3 --variants $VAR > "$ROOT/gpurun_out/$TAG.out" 2> "$ROOT/gpurun_out/$TAG.err" || { tail -20 "$ROOT/gpurun_out/$TAG.err"; return 1; }
  python3 - "$ROOT/gpurun_out/$TAG/pmc_counter_collection.csv" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rows" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, len(v), sorted(v)[len(v)//2])
PY
}
pass SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
