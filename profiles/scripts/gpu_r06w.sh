# r06w: evidence-gather levels opening the single-workgroup chain (PGM_CHAIN_GATHERS=1, C1: one launch per
# query) against a gather launch + the chain; then the single-query GPU suites
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06w; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for G in 0 1; do
  PGM_CHAIN_GATHERS=$G timeout -k 10 200 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1_${G}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  PGM_CHAIN_GATHERS=$G timeout -k 10 200 python bench.py --workload c2 --steps 400 --warmup 40 --no-cpu-baseline > $O/c2_${G}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/c2_${G}_$rep.json')); e=json.load(open('$O/c1_${G}_$rep.json'))
print('gathers $G', 'c1', round(e['value']*1e6,2), 'us', e['parity'].get('ok'), 'c2', round(d['value']*1e6,2), d['parity'].get('ok'), d.get('launches_per_query'))"
done
done
PGM_CHAIN_GATHERS=1 timeout -k 10 300 python -u tools/c1_programs.py > $O/c1_programs.txt 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
tail -1 $O/c1_programs.txt
timeout -k 10 900 python -u -m pytest tests/test_inference_gpu.py tests/test_plan_gpu.py tests/test_compat_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
