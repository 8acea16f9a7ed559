# C3 specialised row kernel: nontemporal marginal stores (PGM_ROWS_JIT_NT) A/B, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PGM_ROWS_JIT_NT=1 timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -m gpu -x -q -k specialised --timeout 120 --timeout-method thread > gpurun_out/pytest_nt.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_nt.log; exit 1; }
tail -1 gpurun_out/pytest_nt.log
for V in 0 1 0 1 0 1; do
  PGM_ROWS_JIT_NT=$V timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 --warmup 10 > gpurun_out/c3nt.json 2> gpurun_out/c3nt.err || { tail gpurun_out/c3nt.err; exit 1; }
  echo "C3 NT=$V $(python -c "import json; d=json.load(open('gpurun_out/c3nt.json')); print(round(d['value']/1e9,2), 'G rows/s', round(d['roofline']['kernel_ms']*1e3,3), 'us/launch', round(d['roofline']['frac'],3))")"
done
