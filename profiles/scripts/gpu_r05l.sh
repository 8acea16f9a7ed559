# r05l: BP update ratio stored by the parent's finalising pass (PGM_PRODN_MDIV): BP parity, C4 A/B
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05l
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "bp or belief or pathfinder or product_n or marginal or calibrat or markov or factor_graph or munin_belief" > gpurun_out/r05l/pytest_bp.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05l/pytest_bp.log; exit 1; }
tail -3 gpurun_out/r05l/pytest_bp.log
for i in 1 2; do for X in 0 1; do for R in 4000 1000; do
  PGM_BP_RATIO=$X timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05l/c4_${X}_${R}_$i.json 2> gpurun_out/r05l/c4.err || { tail -20 gpurun_out/r05l/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05l/c4_${X}_${R}_$i.json')); print('ratio=$X', $R, round(d['value']/1e6,4), 'M/s', d['parity']['ok'], round(d['executed_step_bytes_per_calibration']/1e6,3), 'MB')"
done; done; done
