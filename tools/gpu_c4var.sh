set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_c4.log; exit 1; }
tail -1 gpurun_out/pytest_c4.log
for R in 1000 4000; do
timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 5 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail gpurun_out/c4.err; exit 1; }
echo "rows=$R $(python -c "import json; d=json.load(open('gpurun_out/c4.json')); print(d['value'], d['ms_per_step'], d['achieved_GBps'])")"
done
timeout -k 10 120 python tools/program_steps.py c4 1000 > gpurun_out/steps_c4.txt 2>&1; head -12 gpurun_out/steps_c4.txt | cut -c1-150
