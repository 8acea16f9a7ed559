# batched contraction output pairs (16-B): parity, C4 at 1000/4000 (PGM_NO_ROWS2=1 disables all 16-B row forms: not used here)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cp.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_cp.log; exit 1; }
tail -1 gpurun_out/pytest_cp.log
for R in 1000 4000; do
  timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/c4cp_$R.json 2> gpurun_out/c4cp.err || { tail gpurun_out/c4cp.err; exit 1; }
  echo "C4 R=$R $(python -c "import json; d=json.load(open('gpurun_out/c4cp_$R.json')); print(round(d['value']), round(d['ms_per_step'],3), round(d['achieved_GBps']))")"
done
timeout -k 10 120 python tools/program_steps.py c4 1000 > gpurun_out/steps_c4cp_1000.txt 2>&1; head -14 gpurun_out/steps_c4cp_1000.txt | cut -c1-150
