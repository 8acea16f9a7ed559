# round 3 checkpoint: full GPU suite, smoke, default bench line, rocprof trace/stats + PMC of the default C3 command
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03o}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_plan_gpu.py -k "direct" > gpurun_out/${TAG}_pytest_dq.log 2>&1 || { echo dq tests failed; tail -40 gpurun_out/${TAG}_pytest_dq.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_dq.log
for R in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench_direct20_$R.json 2> gpurun_out/${TAG}_bench_direct20_$R.err || { tail -30 gpurun_out/${TAG}_bench_direct20_$R.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_direct20_$R.json')); r=d['roofline']; print('direct20', round(d['value']/1e9,2), r['frac'], r['frac_wall'])"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail -30 gpurun_out/${TAG}_bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); r=d['roofline']; print(d['value'], d['steps'], r['frac'], r['frac_wall'], r['kernel_ms'], (d.get('api_e2e') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))"
bash tools/gpu_profile.sh $TAG --steps 20 --warmup 5 --no-api-e2e
