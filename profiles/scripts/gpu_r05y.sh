# r05y: C4 with 1 / 2 / 3 calibration batches in flight (own schedules and streams)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05y
export TMPDIR=/tmp
for i in 1 2; do for K in 1 2 3; do for R in 1000 4000; do
  timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 30 --warmup 3 --c4-inflight $K > gpurun_out/r05y/c4_${K}_${R}_$i.json 2> gpurun_out/r05y/c4.err || { tail -20 gpurun_out/r05y/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05y/c4_${K}_${R}_$i.json')); print('inflight=$K', $R, round(d['value']/1e6,4), 'M/s', d['parity']['ok'])"
done; done; done
