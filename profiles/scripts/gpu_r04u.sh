# round 4: blocks per non-reducing batch job (PGM_BATCH_MAX_BLOCKS_PRODUCT 256 = r04p / 1,024 default / 4,096) on C2 /
# C1 / C4 with the tail chain on (the new default), plus the parity suites at the widest setting
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04u}
PGM_BATCH_MAX_BLOCKS_PRODUCT=4096 timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_inference_gpu.py \
  tests/test_factor_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
ab() {  # label workload env -- args
  local L=$1 W=$2 E=$3; shift 4
  env $E timeout -k 10 300 python bench.py --workload $W "$@" --no-cpu-baseline > gpurun_out/${TAG}_${W}_${L}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${L}_$R.json')); v=d['value']; print('$W $L', round(v*1e3,4) if v < 1 else round(v), round(d.get('ms_per_step', 0) or 0, 3))"
}
for R in 1 2; do
  for W in c2 c1; do
    ab p256 $W PGM_BATCH_MAX_BLOCKS_PRODUCT=256 -- --steps 200 --warmup 20
    ab p1024 $W PGM_NOTHING=1 -- --steps 200 --warmup 20
    ab p4096 $W PGM_BATCH_MAX_BLOCKS_PRODUCT=4096 -- --steps 200 --warmup 20
  done
done
R=1
ab p256 c4 PGM_BATCH_MAX_BLOCKS_PRODUCT=256 -- --rows 4000 --steps 20 --warmup 3
ab p1024 c4 PGM_NOTHING=1 -- --rows 4000 --steps 20 --warmup 3
ab p256 c4 PGM_BATCH_MAX_BLOCKS_PRODUCT=256 -- --rows 1000 --steps 20 --warmup 3
ab p1024 c4 PGM_NOTHING=1 -- --rows 1000 --steps 20 --warmup 3
