# r06at: C4's smallest steps specialised too (PGM_PM_MIN_ENTRIES / PGM_PM_PREFER_MIN 4,096 vs 16,384), so they join
# their level's merged launch instead of running as generic kernels: C4 4,000 / 1,000 rows, BP GPU tests with it
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06at; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for M in 16384 4096; do
  PGM_PM_MIN_ENTRIES=$M PGM_PM_PREFER_MIN=$M timeout -k 10 300 python bench.py --workload c4 --rows 4000 --steps 20 --warmup 3 --c4-inflight 1 --no-cpu-baseline > $O/c4_${M}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  PGM_PM_MIN_ENTRIES=$M PGM_PM_PREFER_MIN=$M timeout -k 10 300 python bench.py --workload c4 --rows 1000 --steps 20 --warmup 3 --c4-inflight 1 --no-cpu-baseline > $O/c4k_${M}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/c4_${M}_$rep.json')); e=json.load(open('$O/c4k_${M}_$rep.json'))
print('min $M', '4000', round(d['value']/1e6,4), d['parity'].get('ok'), '1000', round(e['value']/1e6,4), e['parity'].get('ok'))"
done
done
PGM_PM_MIN_ENTRIES=4096 PGM_PM_PREFER_MIN=4096 timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bp or calibrate or pathfinder or belief" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
