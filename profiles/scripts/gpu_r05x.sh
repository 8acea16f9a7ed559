# r05x: inference / plan suites after the speculative direct path and the wide-column cache; api_e2e
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05x
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_plan_gpu.py tests/test_compat_gpu.py > gpurun_out/r05x/t0.log 2>&1 || { tail -40 gpurun_out/r05x/t0.log; exit 1; }
tail -2 gpurun_out/r05x/t0.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-c5 --no-cpu-baseline --no-ring-roofline > gpurun_out/r05x/c3_$i.json 2> gpurun_out/r05x/c3.err || { tail -20 gpurun_out/r05x/c3.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05x/c3_$i.json')); print('c3', round(d['value']/1e9,2), 'G; api_e2e', round(d['api_e2e']['value']/1e6,2), 'M rows/s', round(d['api_e2e']['seconds']*1e3,3), 'ms')"
done
