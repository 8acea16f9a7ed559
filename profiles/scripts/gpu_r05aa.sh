# r05aa: fused plans whose joint is not fused take the steps program through query_one (C1)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05aa
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_plan_gpu.py -k "alarm or query or thread or compiled or direct" > gpurun_out/r05aa/t0.log 2>&1 || { tail -40 gpurun_out/r05aa/t0.log; exit 1; }
tail -2 gpurun_out/r05aa/t0.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c1 --steps 300 --warmup 30 > gpurun_out/r05aa/c1_$i.json 2> gpurun_out/r05aa/c1.err || { tail -20 gpurun_out/r05aa/c1.err; exit 1; }
  python -c "import json; e=json.load(open('gpurun_out/r05aa/c1_$i.json')); print('c1', round(e['value']*1e3,4), 'ms/query; cpu', e.get('cpu_baseline',{}).get('value'))"
done
