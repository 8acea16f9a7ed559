# round 4: lanes per output of batched contractions (PGM_BATCH_LANES 4,096 default / 32,768 / 131,072) on C2 /
# C1 / C4 with the tail chain on (the new default), plus the parity suites at the widest setting
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04p}
PGM_BATCH_LANES=131072 timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_inference_gpu.py \
  tests/test_factor_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
ab() {  # label workload env -- args
  local L=$1 W=$2 E=$3; shift 4
  env $E timeout -k 10 300 python bench.py --workload $W "$@" --no-cpu-baseline > gpurun_out/${TAG}_${W}_${L}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${L}_$R.json')); v=d['value']; print('$W $L', round(v*1e3,4) if v < 1 else round(v), round(d.get('ms_per_step', 0) or 0, 3))"
}
for R in 1 2; do
  for W in c2 c1; do
    ab l4k $W PGM_NOTHING=1 -- --steps 200 --warmup 20
    ab l32k $W PGM_BATCH_LANES=32768 -- --steps 200 --warmup 20
    ab l128k $W PGM_BATCH_LANES=131072 -- --steps 200 --warmup 20
  done
done
R=1
ab l4k c4 PGM_NOTHING=1 -- --rows 4000 --steps 20 --warmup 3
ab l128k c4 PGM_BATCH_LANES=131072 -- --rows 4000 --steps 20 --warmup 3
ab l4k c4 PGM_NOTHING=1 -- --rows 1000 --steps 20 --warmup 3
ab l128k c4 PGM_BATCH_LANES=131072 -- --rows 1000 --steps 20 --warmup 3
