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
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_kernels_gpu.py -k block_order_knobs > gpurun_out/${TAG}_knobs.log 2>&1; rc=$?; tail -8 gpurun_out/${TAG}_knobs.log; [ $rc -le 1 ] || exit 1
for R in 1 2; do
  for ROWS in 4000 1000; do
    c4 default $ROWS PGM_NOTHING=1
    c4 xpart1 $ROWS PGM_PM_XPART=1
    c4 xpart2 $ROWS PGM_PM_XPART=2
    c4 xcd2 $ROWS PGM_PM_XCD=2
    c4 xcd2xpart2 $ROWS PGM_PM_XCD=2 PGM_PM_XPART=2
  done
done
