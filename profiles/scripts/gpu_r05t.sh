# r05t: direct AQL chain with a completion signal on the last packet only (C1 / C2 A/B, parity)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05t
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "direct_chain or threads" > gpurun_out/r05t/t0.log 2>&1 || { tail -40 gpurun_out/r05t/t0.log; exit 1; }
tail -3 gpurun_out/r05t/t0.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05t/c2_${name}_$i.json 2> gpurun_out/r05t/c2.err || { tail -20 gpurun_out/r05t/c2.err; return 1; }
  env "$@" timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 20 > gpurun_out/r05t/c1_${name}_$i.json 2> gpurun_out/r05t/c1.err || { tail -20 gpurun_out/r05t/c1.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05t/c2_${name}_$i.json')); e=json.load(open('gpurun_out/r05t/c1_${name}_$i.json')); print('$name c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
}
for i in 1 2; do
  run graph PGM_QUERY_DIRECT=0 || exit 1
  run lastsig PGM_QUERY_DIRECT=1 || exit 1
  run allsig PGM_DQ_CHAIN_SIG=1 || exit 1
  run lastsig_rel0 PGM_DQ_CHAIN_REL=0 || exit 1
done
