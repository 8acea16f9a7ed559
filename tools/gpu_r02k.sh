set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py tests/test_plan_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ing.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_ing.log; exit 1; }
tail -1 gpurun_out/pytest_ing.log
timeout -k 10 600 python tools/e2e_predict.py 100000 > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -30 gpurun_out/e2e.err; exit 1; }
cat gpurun_out/e2e.json
