# r05n: compile-time chain tuning (chain vs one launch per level, graph-timed) on C1 / C2
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05n
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "chain or specialised" > gpurun_out/r05n/t1.log 2>&1 || { tail -30 gpurun_out/r05n/t1.log; exit 1; }
tail -3 gpurun_out/r05n/t1.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "alarm or munin or c1 or c2" > gpurun_out/r05n/t2.log 2>&1 || { tail -30 gpurun_out/r05n/t2.log; exit 1; }
tail -3 gpurun_out/r05n/t2.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05n/c2_$i.json 2> gpurun_out/r05n/c2.err || { tail -20 gpurun_out/r05n/c2.err; exit 1; }
  timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 20 > gpurun_out/r05n/c1_$i.json 2> gpurun_out/r05n/c1.err || { tail -20 gpurun_out/r05n/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05n/c2_$i.json')); e=json.load(open('gpurun_out/r05n/c1_$i.json')); print('c2', round(d['value']*1e3,4), d['chain_tuning'], d['first_query_s'], 'c1', round(e['value']*1e3,4), e['chain_tuning'], e['first_query_s'], d['parity']['ok'])"
done
