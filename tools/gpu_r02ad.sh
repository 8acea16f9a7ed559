# specialised product+marginal kernel: knob combinations at 4000 and 1000 rows (two passes each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
run() { # label rows env...
  local lab=$1 rows=$2; shift 2
  env "$@" $T 300 python -u bench.py --workload c4 --rows $rows --steps 30 --warmup 3 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c4_$lab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c4_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']), round(d['ms_per_step'],3))"
}
for pass in 1 2; do
run jit_$pass 4000 PGM_PM_JIT=1
run xi1_$pass 4000 PGM_PM_XI=1
run xi1nt_$pass 4000 PGM_PM_XI=1 PGM_PM_NT=1
run xi1ntxcd_$pass 4000 PGM_PM_XI=1 PGM_PM_NT=1 PGM_PM_XCD=1
run xi1xcd_$pass 4000 PGM_PM_XI=1 PGM_PM_XCD=1
run ntxcd_$pass 4000 PGM_PM_NT=1 PGM_PM_XCD=1
done
run k1000_base 1000 PGM_PM_JIT=0
run k1000_jit 1000 PGM_PM_JIT=1
run k1000_xi1nt 1000 PGM_PM_XI=1 PGM_PM_NT=1
run k1000_min 1000 PGM_PM_JIT_MIN=262144
run k1000_min_nt 1000 PGM_PM_JIT_MIN=262144 PGM_PM_NT=1
run k4000_min 4000 PGM_PM_JIT_MIN=262144
