# r05ah: single-query host path trimmed (bound programs skip the queue lookup; env scan once)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05ah
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "direct_chain or threads or munin_c2" > gpurun_out/r05ah/t0.log 2>&1 || { tail -40 gpurun_out/r05ah/t0.log; exit 1; }
tail -1 gpurun_out/r05ah/t0.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05ah/c2_$i.json 2> gpurun_out/r05ah/c2.err || { tail -20 gpurun_out/r05ah/c2.err; exit 1; }
  timeout -k 10 300 python -u bench.py --workload c1 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r05ah/c1_$i.json 2> gpurun_out/r05ah/c1.err || { tail -20 gpurun_out/r05ah/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05ah/c2_$i.json')); e=json.load(open('gpurun_out/r05ah/c1_$i.json')); print('c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
done
