set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -k "two_marginals or product_n or bp or pathfinder or jt3 or max or munin_belief" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pm2.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_pm2.log; exit 1; }
tail -1 gpurun_out/pytest_pm2.log
run() { # label rows env...
  local lab=$1 rows=$2; shift 2
  env "$@" $T 300 python -u bench.py --workload c4 --rows $rows --steps 30 --warmup 3 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c4_$lab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c4_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']), round(d['ms_per_step'],3))"
}
run pm2_4000 4000
run nopm2_4000 4000 PGM_PM2=0
run pm2_1000 1000
run nopm2_1000 1000 PGM_PM2=0
LEVELS=1 TOP=0 $T 300 python -u tools/program_steps.py c4 4000 > gpurun_out/c4_levels_4000p.txt 2>&1 || { tail -30 gpurun_out/c4_levels_4000p.txt; exit 1; }
head -3 gpurun_out/c4_levels_4000p.txt
