# C3 specialised row kernel: workgroup size sweep (PGM_ROWS_JIT_WG) at 100k / 1M rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for WG in 64 128 256; do
  PGM_ROWS_JIT_WG=$WG timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -m gpu -x -q -k specialised --timeout 120 --timeout-method thread > gpurun_out/pytest_wg$WG.log 2>&1 || { echo "tests failed WG=$WG"; tail -30 gpurun_out/pytest_wg$WG.log; exit 1; }
  echo "WG=$WG $(tail -1 gpurun_out/pytest_wg$WG.log)"
  PGM_ROWS_JIT_WG=$WG timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 --warmup 10 > gpurun_out/c3wg$WG.json 2> gpurun_out/c3wg$WG.err || { tail gpurun_out/c3wg$WG.err; exit 1; }
  echo "C3 WG=$WG $(python -c "import json; d=json.load(open('gpurun_out/c3wg$WG.json')); print(round(d['value']/1e9,2), 'G rows/s', round(d['roofline']['kernel_ms']*1e3,3), 'us/launch', round(d['roofline']['frac'],3))")"
  PGM_ROWS_JIT_WG=$WG timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 10 --rows 1000000 > gpurun_out/c3wg${WG}_1m.json 2> gpurun_out/c3wg$WG.err || { tail gpurun_out/c3wg$WG.err; exit 1; }
  echo "C3 1M WG=$WG $(python -c "import json; d=json.load(open('gpurun_out/c3wg${WG}_1m.json')); print(round(d['value']/1e9,2), 'G rows/s', round(d['roofline']['kernel_ms']*1e3,3), 'us/launch', round(d['roofline']['frac'],3))")"
done
