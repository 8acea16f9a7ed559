set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -k "product_n or bp or pathfinder or jt3 or disk_cache or max" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_pm.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_pm.log; exit 1; }
tail -1 gpurun_out/pytest_pm.log
run() { # label rows env...
  local lab=$1 rows=$2; shift 2
  env "$@" $T 300 python -u bench.py --workload c4 --rows $rows --steps 30 --warmup 3 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c4_$lab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c4_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']), round(d['ms_per_step'],3))"
}
run all4000 4000
run all1000 1000
LEVELS=1 TOP=0 $T 300 python -u tools/program_steps.py c4 4000 > gpurun_out/c4_levels_4000n.txt 2>&1 || { tail -30 gpurun_out/c4_levels_4000n.txt; exit 1; }
head -3 gpurun_out/c4_levels_4000n.txt
