set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
run() { # label rows env...
  local lab=$1 rows=$2; shift 2
  env "$@" $T 300 python -u bench.py --workload c4 --rows $rows --steps 30 --warmup 3 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c4_$lab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c4_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']), round(d['ms_per_step'],3))"
}
$T 300 python -u tools/pm_build_time.py 4000 2>&1 | grep rows
PGM_PM_JIT_MIN=65536 $T 300 python -u tools/pm_build_time.py 1000 2>&1 | grep rows
$T 300 python -u tools/pm_build_time.py 1000 2>&1 | grep rows
run d4000 4000
run d1000 1000
run m64k_1000 1000 PGM_PM_JIT_MIN=65536
run m64k_4000 4000 PGM_PM_JIT_MIN=65536
run m16k_1000 1000 PGM_PM_JIT_MIN=16384
