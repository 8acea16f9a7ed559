# r05z: C4 in-flight lanes in the library (BatchedJunctionTree inflight): tests, bench 1 / 2 in flight
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05z
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "pathfinder or bp or belief" > gpurun_out/r05z/t0.log 2>&1 || { tail -40 gpurun_out/r05z/t0.log; exit 1; }
tail -2 gpurun_out/r05z/t0.log
for i in 1 2; do for K in 2 1; do for R in 4000 1000; do
  timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 --c4-inflight $K > gpurun_out/r05z/c4_${K}_${R}_$i.json 2> gpurun_out/r05z/c4.err || { tail -20 gpurun_out/r05z/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05z/c4_${K}_${R}_$i.json')); print('inflight=$K', $R, round(d['value']/1e6,4), 'M/s', d['parity']['ok'])"
done; done; done
