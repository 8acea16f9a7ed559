# r05r: compiled single queries as one AQL chain on a user-mode queue (Program.bind_direct) vs graph replay
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05r
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "direct_chain" > gpurun_out/r05r/t0.log 2>&1 || { tail -40 gpurun_out/r05r/t0.log; exit 1; }
tail -3 gpurun_out/r05r/t0.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_plan_gpu.py > gpurun_out/r05r/t1.log 2>&1 || { tail -40 gpurun_out/r05r/t1.log; exit 1; }
tail -3 gpurun_out/r05r/t1.log
for i in 1 2; do for X in 1 0; do
  PGM_QUERY_DIRECT=$X timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05r/c2_${X}_$i.json 2> gpurun_out/r05r/c2.err || { tail -20 gpurun_out/r05r/c2.err; exit 1; }
  PGM_QUERY_DIRECT=$X timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 20 > gpurun_out/r05r/c1_${X}_$i.json 2> gpurun_out/r05r/c1.err || { tail -20 gpurun_out/r05r/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05r/c2_${X}_$i.json')); e=json.load(open('gpurun_out/r05r/c1_${X}_$i.json')); print('direct=$X c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
done; done
