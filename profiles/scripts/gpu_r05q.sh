# r05q: row-chunk position in the specialised steps' block decode (C4 A/B): fastest (r02-r05), just above the
# XCD-partitioned kept dim, slowest
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05q
export TMPDIR=/tmp
PGM_PM_XBPOS=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "product_n or bp_levelled or pathfinder_bp or two_marginals" > gpurun_out/r05q/pytest.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05q/pytest.log; exit 1; }
tail -3 gpurun_out/r05q/pytest.log
run() {  # name, env...
  local name=$1; shift
  for R in 4000 1000; do
    env "$@" timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05q/c4_${name}_${R}_$i.json 2> gpurun_out/r05q/c4.err || { tail -20 gpurun_out/r05q/c4.err; return 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05q/c4_${name}_${R}_$i.json')); print('$name', $R, round(d['value']/1e6,4), 'M/s', d['parity']['ok'])"
  done
}
for i in 1 2; do
  run fast PGM_PM_XBPOS=0 || exit 1
  run mid PGM_PM_XBPOS=1 || exit 1
  run slow PGM_PM_XBPOS=2 || exit 1
done
PGM_PM_XBPOS=1 timeout -k 10 300 python -u tools/c4_dump.py gpurun_out/r05q/d4000 > gpurun_out/r05q/d4000.log 2>&1 || { tail -20 gpurun_out/r05q/d4000.log; exit 1; }
