# r06e: the single-query fast path (_FastQuery: codes as bytes straight into the host codes buffer) and
# the cached column checks / result columns of the DataFrame API: inference + plan GPU suites, then
# C2's split, the API stage profile, and the C1 / C2 lines
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_inference_gpu.py tests/test_plan_gpu.py tests/test_compat_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python tools/c2_split.py 2000 > $O/c2_split.json 2> $O/c2_split.err || { tail -20 $O/c2_split.err; exit 1; }
cat $O/c2_split.json
timeout -k 10 200 python tools/e2e_stages.py 100000 20 > $O/e2e_stages.txt 2> $O/e2e_stages.err || { tail -20 $O/e2e_stages.err; exit 1; }
head -6 $O/e2e_stages.txt
timeout -k 10 120 python bench.py --workload c1 --steps 300 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
timeout -k 10 120 python bench.py --workload c2 --steps 1000 --warmup 40 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python -c "
import json
for k in ('c1','c2'):
    d=json.load(open('$O/'+k+'.json')); print(k, round(d['value']*1e6,2), 'us/query parity', d['parity']['ok'], 'cpu', d.get('cpu_baseline',{}).get('value'))"
