# round 4: C4 kept-dim decode order A/B (PGM_PM_XPART 0 / 1 / 2, PGM_PM_KREV=1 for reference; PGM_PM_XCD=2
# bijective XCD grouping for block counts not divisible by 8):
# calibrations/s at 1,000 and 4,000 rows (two repeats, interleaved), then FETCH_SIZE per step of the
# 4,000-row schedule for XPART 0 / 1 / 2 (separate --pmc passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04c}
c4() {  # label rows env...
  local L=$1 ROWS=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json')); print('c4 $ROWS $L', round(d['value']), round(d['ms_per_step'],3), 'ms')"
}
# C5 MAP host-delivery loop under a kernel + memory-copy trace (where do 0.3 ms per step go?)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$ROOT/gpurun_out/${TAG}_c5trace" -o t --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c5 --c5-output map --steps 20 --warmup 5 > "$ROOT/gpurun_out/${TAG}_c5trace.json" 2> "$ROOT/gpurun_out/${TAG}_c5trace.err") \
  || { echo "c5 trace failed"; tail -5 gpurun_out/${TAG}_c5trace.err; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_kernels_gpu.py -k block_order_knobs > gpurun_out/${TAG}_knobs.log 2>&1; rc=$?; tail -8 gpurun_out/${TAG}_knobs.log; [ $rc -le 1 ] || exit 1
for R in 1; do
  for ROWS in 4000 1000; do
    c4 default $ROWS PGM_NOTHING=1
    c4 xpart1 $ROWS PGM_PM_XPART=1
    c4 xpart2 $ROWS PGM_PM_XPART=2
    c4 xcd2 $ROWS PGM_PM_XCD=2
    c4 xcd2xpart2 $ROWS PGM_PM_XCD=2 PGM_PM_XPART=2
  done
done
cd /tmp && export TMPDIR=/tmp
for X in 0 1 2; do
  for C in FETCH_SIZE WRITE_SIZE; do
    PGM_PM_XCD=$([ $X -eq 2 ] && echo 2 || echo 1) PGM_PM_XPART=$X timeout -s KILL 120 rocprofv3 --pmc $C -d "$ROOT/gpurun_out/${TAG}_pmc_${X}_$C" -o p --output-format csv -- \
      python3 "$ROOT/tools/c4_step_pmc.py" run "$ROOT/gpurun_out/${TAG}_pmc_meta_$X.json" > "$ROOT/gpurun_out/${TAG}_pmc_${X}_${C}.log" 2>&1 \
      || { echo "pmc $X $C failed"; tail -5 "$ROOT/gpurun_out/${TAG}_pmc_${X}_${C}.log"; exit 1; }
  done
  python3 "$ROOT/tools/c4_step_pmc.py" summarize "$ROOT/gpurun_out/${TAG}_pmc_meta_$X.json" "$ROOT/gpurun_out/${TAG}_pmc_${X}_FETCH_SIZE" \
    "$ROOT/gpurun_out/${TAG}_pmc_${X}_WRITE_SIZE" > "$ROOT/gpurun_out/${TAG}_pmc_summary_$X.json"
  python3 -c "import json; d=json.load(open('$ROOT/gpurun_out/${TAG}_pmc_summary_$X.json')); print('xpart $X fetch GB', round(d['fetch_bytes_x2']/1e9,2), 'write GB', round(d['write_bytes']/1e9,2), 'ratio floor', round(d['ratio_to_floor'],2)); [print('  ', t['step'], round(t['fetch_MB_x2']), round(t['write_MB']), round(t['alg_MB']), t['note'][:70]) for t in d['top'][:6]]"
done
cd "$ROOT"
c2() {  # label workload env...
  local L=$1 W=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_${W}_${L}_$R.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${L}_$R.json')); print('$W $L', round(d['value']*1e3,4), 'ms/query')"
}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_kernels_gpu.py -k block_order_knobs > gpurun_out/${TAG}_knobs.log 2>&1; rc=$?; tail -8 gpurun_out/${TAG}_knobs.log; [ $rc -le 1 ] || exit 1
for R in 1; do
  c2 default c2 PGM_NOTHING=1
  c2 onejob c2 PGM_ONE_JOB_AS_BATCH=1
  c2 default c1 PGM_NOTHING=1
  c2 onejob c1 PGM_ONE_JOB_AS_BATCH=1
done
cd "$ROOT"; timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps.txt 2>&1 && head -60 gpurun_out/${TAG}_c2_steps.txt
