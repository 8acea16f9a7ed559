set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_compat_gpu.py tests/test_inference_gpu.py -k "compat or hip_backend or categorical" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_compat.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_compat.log; exit 1; }
tail -8 gpurun_out/pytest_compat.log
