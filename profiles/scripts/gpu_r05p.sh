# r05p: merged specialised launches: tree dispatch vs the linear chain, waves-per-EU bound (C4 A/B)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05p
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "product_n or bp_levelled or pathfinder_bp" > gpurun_out/r05p/pytest.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05p/pytest.log; exit 1; }
tail -3 gpurun_out/r05p/pytest.log
run() {  # name, env...
  local name=$1; shift
  for R in 4000 1000; do
    env "$@" timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05p/c4_${name}_${R}_$i.json 2> gpurun_out/r05p/c4.err || { tail -20 gpurun_out/r05p/c4.err; return 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05p/c4_${name}_${R}_$i.json')); print('$name', $R, round(d['value']/1e6,4), 'M/s', d['parity']['ok'])"
  done
}
for i in 1 2; do
  run tree PGM_X=0 || exit 1
  run linear PGM_PM_LINEAR=1 || exit 1
  run wpe5 PGM_PM_WPE=5 || exit 1
  run wpe6 PGM_PM_WPE=6 || exit 1
  run wpe8 PGM_PM_WPE=8 || exit 1
done
