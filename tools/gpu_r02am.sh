set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
run() { # label rows env...
  local lab=$1 rows=$2; shift 2
  env "$@" $T 300 python -u bench.py --workload c4 --rows $rows --steps 30 --warmup 3 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c4_$lab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c4_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']), round(d['ms_per_step'],3))"
}
run d4000 4000
run d1000 1000
