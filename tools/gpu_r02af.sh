set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_all.log; exit 1; }
tail -3 gpurun_out/pytest_all.log
