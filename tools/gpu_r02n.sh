set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py -k "stochastic or categorical or late_edits" -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_sto.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_sto.log; exit 1; }
tail -8 gpurun_out/pytest_sto.log
