# SQ instruction-mix counters for the fused row kernel at a given batch size.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"; TAG=${1:-sq}; ROWS=${2:-1000000}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace -d "$ROOT/gpurun_out/$TAG" -o pmc --output-format csv -- \
  python3 "$ROOT/tools/rows_sweep.py" --rows $ROWS --reps 3 > "$ROOT/gpurun_out/$TAG.out" 2> "$ROOT/gpurun_out/$TAG.err" || { tail -20 "$ROOT/gpurun_out/$TAG.err"; exit 1; }
python3 - "$ROOT/gpurun_out/$TAG/pmc_counter_collection.csv" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rows" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, len(v), sorted(v)[len(v)//2])
PY
