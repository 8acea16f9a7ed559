# r06ao: single-pass evidence mapping in _FastQuery: inference / compat GPU suites, C1 / C2 twice
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ao; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py tests/test_compat_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  timeout -k 10 200 python bench.py --workload c2 --steps 400 --warmup 40 --no-cpu-baseline > $O/c2_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/c2_$rep.json')); e=json.load(open('$O/c1_$rep.json'))
print('c1', round(e['value']*1e6,2), 'us', e['parity'].get('ok'), 'c2', round(d['value']*1e6,2), d['parity'].get('ok'), d.get('launches_per_query'))"
done
timeout -k 10 300 python -u tools/query_split.py 200 > $O/split.txt 2> $O/split.err || { tail -30 $O/split.err; exit 1; }
tail -1 $O/split.txt
