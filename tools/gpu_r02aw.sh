set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py -k "bench_size" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bs.log 2>&1 || { echo failed; tail -60 gpurun_out/pytest_bs.log; exit 1; }
tail -1 gpurun_out/pytest_bs.log
