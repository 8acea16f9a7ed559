set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py -k "munin_belief" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_mbp.log 2>&1 || { echo failed; tail -40 gpurun_out/pytest_mbp.log; exit 1; }
tail -1 gpurun_out/pytest_mbp.log
