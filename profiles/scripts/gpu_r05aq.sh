# r05aq: chain length re-checked after the single-query routing and fence changes
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05aq
export TMPDIR=/tmp
for i in 1 2; do for X in 4 8 16; do
  PGM_WG_CHAIN_BLOCKS=$X timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05aq/c2_${X}_$i.json 2> gpurun_out/r05aq/c2.err || { tail -20 gpurun_out/r05aq/c2.err; exit 1; }
  PGM_WG_CHAIN_BLOCKS=$X timeout -k 10 300 python -u bench.py --workload c1 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r05aq/c1_${X}_$i.json 2> gpurun_out/r05aq/c1.err || { tail -20 gpurun_out/r05aq/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05aq/c2_${X}_$i.json')); e=json.load(open('gpurun_out/r05aq/c1_${X}_$i.json')); print('chain<=$X c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
done; done
