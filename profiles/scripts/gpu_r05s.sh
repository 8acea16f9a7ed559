# r05s: direct AQL chain for compiled queries: fences, doorbell, queue profiling (C1 / C2 A/B)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05s
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05s/c2_${name}_$i.json 2> gpurun_out/r05s/c2.err || { tail -20 gpurun_out/r05s/c2.err; return 1; }
  env "$@" timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 20 > gpurun_out/r05s/c1_${name}_$i.json 2> gpurun_out/r05s/c1.err || { tail -20 gpurun_out/r05s/c1.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05s/c2_${name}_$i.json')); e=json.load(open('gpurun_out/r05s/c1_${name}_$i.json')); print('$name c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
}
for i in 1 2; do
  run graph PGM_QUERY_DIRECT=0 || exit 1
  run agent PGM_QUERY_DIRECT=1 || exit 1
  run acq0 PGM_DQ_CHAIN_ACQ=0 || exit 1
  run rel0 PGM_DQ_CHAIN_REL=0 || exit 1
  run sys PGM_DQ_CHAIN_ACQ=2 PGM_DQ_CHAIN_REL=2 || exit 1
  run db PGM_DQ_CHAIN_DB=1 || exit 1
  run prof PGM_DQ_QPROF=1 || exit 1
done
