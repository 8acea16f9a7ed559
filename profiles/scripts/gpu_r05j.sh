# r05j: full GPU suite + smoke after the specialised contraction batches
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05j
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05j/pytest_gpu.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05j/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r05j/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05j/smoke.log 2>&1 || { tail -30 gpurun_out/r05j/smoke.log; exit 1; }
tail -1 gpurun_out/r05j/smoke.log
