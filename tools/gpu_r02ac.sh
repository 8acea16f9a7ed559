# specialised product+marginal kernel: parity tests, then C4 A/B over the knobs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_kernels_gpu.py -k "product_n_marginal or bp_fused" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_pm.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_pm.log; exit 1; }
tail -1 gpurun_out/pytest_pm.log
run() { # label env...
  local lab=$1; shift
  env "$@" $T 300 python -u bench.py --workload c4 --rows 4000 --steps 20 --warmup 3 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c4_$lab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c4_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']), round(d['ms_per_step'],3))"
}
run base PGM_PM_JIT=0
run jit PGM_PM_JIT=1
run jit_xcd PGM_PM_XCD=1
run jit_nt PGM_PM_NT=1
run jit_u4 PGM_PM_UNROLL=4
run jit_u16 PGM_PM_UNROLL=16
run jit_xi1 PGM_PM_XI=1
run jit_xi4 PGM_PM_XI=4
$T 300 python -u tools/program_steps.py c4 4000 > gpurun_out/c4_steps_jit.txt 2>&1 || { tail -20 gpurun_out/c4_steps_jit.txt; exit 1; }
