# r06ae: fusion at 512 Ki / 512 with split n-ary walks as the default: the whole GPU suite, C1 / C2 bench twice
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ae; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  timeout -k 10 200 python bench.py --workload c2 --steps 400 --warmup 40 --no-cpu-baseline > $O/c2_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/c2_$rep.json')); e=json.load(open('$O/c1_$rep.json'))
print('c1', round(e['value']*1e6,2), 'us', e['parity'].get('ok'), 'c2', round(d['value']*1e6,2), d['parity'].get('ok'), d['parity'].get('mass_max_rel_err'), d.get('launches_per_query'))"
done
