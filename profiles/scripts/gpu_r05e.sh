# r05e: C4 with direct child-message operands (MOPS 8): BP / fused-kernel parity, C4 rates, schedule dump
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "bp or belief or pathfinder or product_n or marginal or calibrat or markov or factor_graph" > gpurun_out/r05e/pytest_bp.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05e/pytest_bp.log; exit 1; }
tail -3 gpurun_out/r05e/pytest_bp.log
for R in 4000 1000; do
  for i in 1 2; do
    timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05e/c4_${R}_$i.json 2> gpurun_out/r05e/c4.err || { tail -20 gpurun_out/r05e/c4.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05e/c4_${R}_$i.json')); print($R, round(d['value']/1e6,4), 'M/s', round(d['ms_per_step'],3), 'ms', d['parity']['ok'], d['executed_step_bytes_per_calibration'])"
  done
done
ROWS=4000 timeout -k 10 300 python tools/c4_dump.py gpurun_out/r05e/c4dump > gpurun_out/r05e/c4dump.log 2>&1 || { tail -20 gpurun_out/r05e/c4dump.log; exit 1; }
