# r05aj: C3 queue count 4 vs 5 (20-step driver window and 400 steps)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05aj
export TMPDIR=/tmp
for i in 1 2 3; do for Q in 4 5 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --queues $Q --no-c5 --no-cpu-baseline --no-api-e2e --no-ring-roofline > gpurun_out/r05aj/q${Q}_20_$i.json 2> gpurun_out/r05aj/c3.err || { tail -20 gpurun_out/r05aj/c3.err; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 400 --warmup 20 --queues $Q --no-c5 --no-cpu-baseline --no-api-e2e --no-ring-roofline > gpurun_out/r05aj/q${Q}_400_$i.json 2> gpurun_out/r05aj/c3.err || { tail -20 gpurun_out/r05aj/c3.err; exit 1; }
  python -c "
import json
a=json.load(open('gpurun_out/r05aj/q${Q}_20_$i.json')); b=json.load(open('gpurun_out/r05aj/q${Q}_400_$i.json'))
print('queues=$Q', '20 steps', round(a['value']/1e9,2), 'G frac', round(a['roofline']['frac'],3), '| 400 steps', round(b['value']/1e9,2), 'G frac', round(b['roofline']['frac'],3))"
done; done
