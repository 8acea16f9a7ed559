# C3 row kernel iteration: parity tests, rows sweep, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_c3.log; exit 1; }
tail -2 gpurun_out/pytest_c3.log
for J in 0 1; do
  if [ $J = 1 ]; then export PGM_NO_JIT2=1; fi
  timeout -k 10 120 python tools/rows_sweep.py --rows 100000 1000000 4000000 --reps 200 --variants lds_values map_only torch_fill_floor > gpurun_out/rows_sweep$J.txt 2>&1; echo "NO_JIT2=$J"; grep -o '"rows": [0-9]*\|"variant": "[a-z_]*"\|"kernel_us": [0-9.]*' gpurun_out/rows_sweep$J.txt | paste - - -
  timeout -k 10 300 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/bench_j$J.json 2> gpurun_out/bench_j$J.err || { tail gpurun_out/bench_j$J.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_j$J.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'])"
done
