set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_gemm.log; exit 1; }
tail -1 gpurun_out/pytest_gemm.log
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1; grep -o '"batch": [0-9]*, "M": [0-9]*, "N": [0-9]*, "K": [0-9]*, "gemm_us": [0-9.]*, "gemm_TFLOPs": [0-9.]*' gpurun_out/gemm_bench.txt
timeout -k 10 200 python tools/program_steps.py c2 > gpurun_out/steps_c2.txt 2>&1; head -30 gpurun_out/steps_c2.txt | cut -c1-150
timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print(d['value'], d['achieved'])"
