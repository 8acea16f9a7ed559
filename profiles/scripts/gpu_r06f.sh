# r06f: n-ary contraction jobs (fused contraction paths): kernel tests, fused vs unfused query programs,
# hazards, the query parity suites, then C2's split and the C1 / C2 lines
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "contract_n or fused_query or specialised" > $O/pytest_k.log 2>&1 || { tail -60 $O/pytest_k.log; exit 1; }
tail -3 $O/pytest_k.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hazards_gpu.py tests/test_inference_gpu.py -k "c2 or alarm or munin or hazard or query or bn6 or thread" > $O/pytest_i.log 2>&1 || { tail -60 $O/pytest_i.log; exit 1; }
tail -3 $O/pytest_i.log
timeout -k 10 120 python tools/c2_split.py 2000 > $O/c2_split.json 2> $O/c2_split.err || { tail -20 $O/c2_split.err; exit 1; }
cat $O/c2_split.json
timeout -k 10 120 python bench.py --workload c1 --steps 300 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
timeout -k 10 120 python bench.py --workload c2 --steps 1000 --warmup 40 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python -c "
import json
for k in ('c1','c2'):
    d=json.load(open('$O/'+k+'.json')); print(k, round(d['value']*1e6,2), 'us/query parity', d['parity'], d.get('launches_per_query'), d.get('plan'))"
