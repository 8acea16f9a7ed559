# r05c: full GPU suite + smoke after the r05 knob prune
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05c/pytest_gpu.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05c/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r05c/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05c/smoke.log 2>&1 \
  || { echo smoke failed; tail -30 gpurun_out/r05c/smoke.log; exit 1; }
tail -1 gpurun_out/r05c/smoke.log
timeout -k 10 300 python -u bench.py --workload c2 --steps 200 --warmup 20 > gpurun_out/r05c/c2.json 2> gpurun_out/r05c/c2.err && cat gpurun_out/r05c/c2.json | head -c 400; echo
timeout -k 10 300 python -u bench.py --workload c4 --rows 4000 --steps 10 --warmup 3 > gpurun_out/r05c/c4_4000.json 2> gpurun_out/r05c/c4.err && head -c 300 gpurun_out/r05c/c4_4000.json; echo
timeout -k 10 300 python -u bench.py --workload c4 --rows 1000 --steps 20 --warmup 3 > gpurun_out/r05c/c4_1000.json 2>> gpurun_out/r05c/c4.err && head -c 300 gpurun_out/r05c/c4_1000.json; echo
