set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py -k "edge" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_e.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_e.log; exit 1; }
tail -1 gpurun_out/pytest_e.log
