set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_factor_graph.py -k "bp or BP or calibrat or belief or product_n or jt3 or factor_graph" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_bp.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_bp.log; exit 1; }
tail -1 gpurun_out/pytest_bp.log
for R in 1000 4000; do
timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/c4_$R.json 2> gpurun_out/c4_$R.err || { tail -30 gpurun_out/c4_$R.err; exit 1; }
cat gpurun_out/c4_$R.json
done
timeout -k 10 300 python tools/program_steps.py c4 4000 > gpurun_out/steps_c4_4000.txt 2>&1 || { tail -20 gpurun_out/steps_c4_4000.txt; exit 1; }
head -14 gpurun_out/steps_c4_4000.txt | cut -c1-220
