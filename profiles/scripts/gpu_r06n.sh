# r06n: C4 4,000 rows with up to 64 vs 128 bodies per merged launch (level 1 holds 74 specialised steps),
# the step dump at 128, and the C4 GPU tests
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp
for B in 64 128 64 128; do
  PGM_PM_MERGE_BODIES=$B timeout -k 10 300 python bench.py --workload c4 --rows 4000 --steps 20 --warmup 3 --no-cpu-baseline > $O/c4_$B.json 2>> $O/c4.err \
    || { tail -30 $O/c4.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/c4_$B.json')); print('bodies $B', d['value'], d['ms_per_step'], (d.get('two_in_flight') or {}).get('value'), d.get('launches_per_sweep', d.get('launches')))"
done
ROWS=4000 timeout -k 10 300 python -u tools/c4_dump.py $O/d4000 > $O/d4000.log 2>&1 || { tail -20 $O/d4000.log; exit 1; }
tail -3 $O/d4000.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bp or calibrate or belief or pm_merge or merge" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
