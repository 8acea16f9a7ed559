# round 4: C4 with a longer unroll on steps of few blocks (PGM_PM_UNROLL_SMALL = block threshold), 4,000 and
# 1,000 rows, interleaved, two repeats; parity of the batched-BP tests at one setting
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04z}
PGM_PM_UNROLL_SMALL=4096 timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_inference_gpu.py -k "pathfinder or bp" \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
c4() {  # label rows env
  local L=$1 ROWS=$2 E=$3
  env $E timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json')); print('c4 $ROWS $L', round(d['value']), round(d['ms_per_step'],3), 'ms')"
}
for R in 1 2; do
  for ROWS in 1000 4000; do
    c4 default $ROWS PGM_NOTHING=1
    c4 s1024 $ROWS PGM_PM_UNROLL_SMALL=1024
    c4 s2048 $ROWS PGM_PM_UNROLL_SMALL=2048
    c4 s4096 $ROWS PGM_PM_UNROLL_SMALL=4096
    c4 s16384 $ROWS PGM_PM_UNROLL_SMALL=16384
  done
done
