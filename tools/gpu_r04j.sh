# round 4: blocks per batch job (PGM_BATCH_MAX_BLOCKS 256 / 1024 / 4096): C2 / C1 latency, C4 calibrations/s,
# and parity of the batch paths at the widest setting
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04j}
PGM_BATCH_MAX_BLOCKS=4096 timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_inference_gpu.py \
  -k "batch or c2 or pathfinder or alarm" > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
run() {  # workload blocks extra-args...
  local W=$1 B=$2; shift 2
  PGM_BATCH_MAX_BLOCKS=$B timeout -k 10 300 python bench.py --workload $W "$@" --no-cpu-baseline > gpurun_out/${TAG}_${W}_${B}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${B}_$R.json')); v=d['value']; print('$W blocks $B', round(v*1e3,4) if v < 1 else round(v), d.get('ms_per_step',''))"
}
for R in 1 2; do
  for B in 256 1024 4096; do
    run c2 $B --steps 200 --warmup 20
    run c1 $B --steps 200 --warmup 20
  done
done
for B in 256 4096; do
  R=1 run c4 $B --rows 4000 --steps 20 --warmup 3
done
PGM_BATCH_MAX_BLOCKS=4096 timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps_4096.txt 2>&1 && grep "steps," gpurun_out/${TAG}_c2_steps_4096.txt
