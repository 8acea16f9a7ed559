# C3 row kernel iteration: parity tests, rows sweep, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py tests/test_inference_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_c3.log; exit 1; }
tail -2 gpurun_out/pytest_c3.log
timeout -k 10 120 python tools/rows_sweep.py --rows 100000 1000000 4000000 --variants lds_values map_only torch_fill_floor > gpurun_out/rows_sweep.txt 2>&1; grep -o '"rows": [0-9]*\|"variant": "[a-z_]*"\|"kernel_us": [0-9.]*\|"host_us_per_launch": [0-9.]*' gpurun_out/rows_sweep.txt | paste - - - - 
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail gpurun_out/bench1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench1.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['parity'])"
