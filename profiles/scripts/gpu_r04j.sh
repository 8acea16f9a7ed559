# round 4: C2 / C1 A/B of the contraction kept-dim order (PGM_CONTRACT_ORDER 0 / then-default 1) and of the blocks per
# batch job (PGM_BATCH_MAX_BLOCKS 256 / 1024 / 4096); C4 at the extremes; parity of the contraction and batch
# paths at the new defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04j}
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_inference_gpu.py \
  tests/test_factor_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
run() {  # label workload env... -- args
  local L=$1 W=$2; shift 2
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --workload $W "$@" --no-cpu-baseline > gpurun_out/${TAG}_${W}_${L}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${L}_$R.json')); v=d['value']; print('$W $L', round(v*1e3,4) if v < 1 else round(v), round(d.get('ms_per_step', 0) or 0, 3))"
}
for R in 1 2; do
  for W in c2 c1; do
    run order0 $W PGM_CONTRACT_ORDER=0 -- --steps 200 --warmup 20
    run default $W PGM_NOTHING=1 -- --steps 200 --warmup 20
    run b1024 $W PGM_BATCH_MAX_BLOCKS=1024 -- --steps 200 --warmup 20
    run b4096 $W PGM_BATCH_MAX_BLOCKS=4096 -- --steps 200 --warmup 20
  done
done
R=1
run order0 c4 PGM_CONTRACT_ORDER=0 -- --rows 4000 --steps 20 --warmup 3
run default c4 PGM_NOTHING=1 -- --rows 4000 --steps 20 --warmup 3
run b4096 c4 PGM_BATCH_MAX_BLOCKS=4096 -- --rows 4000 --steps 20 --warmup 3
timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps.txt 2>&1 && grep -A12 "steps," gpurun_out/${TAG}_c2_steps.txt
PGM_CONTRACT_ORDER=0 timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps_order0.txt 2>&1 && grep -A12 "steps," gpurun_out/${TAG}_c2_steps_order0.txt
