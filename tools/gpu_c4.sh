# C4 kernels: parity of the row paths, then C4 bench at 1000/4000 rows and per-step timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_c4.log; exit 1; }
tail -2 gpurun_out/pytest_c4.log
for R in 1000 4000; do
  timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 5 --warmup 1 > gpurun_out/bench_c4_$R.json 2> gpurun_out/bench_c4_$R.err || { tail gpurun_out/bench_c4_$R.err; exit 1; }
  cat gpurun_out/bench_c4_$R.json
done
timeout -k 10 120 python tools/program_steps.py c4 1000 > gpurun_out/steps_c4_1000.txt 2>&1; head -16 gpurun_out/steps_c4_1000.txt | cut -c1-200
