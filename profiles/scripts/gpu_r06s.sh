# r06s: C2 / C1 with the specialised batch kernels' buffer addresses baked in as literals (PGM_CS_BAKE=1)
# against kernel-argument loads (default)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06s; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for K in 0 1; do
  export PGM_CS_BAKE=$K
  timeout -k 10 300 python bench.py --workload c2 --steps 400 --warmup 40 --no-cpu-baseline > $O/c2_${K}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  timeout -k 10 300 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1_${K}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/c2_${K}_$rep.json')); e=json.load(open('$O/c1_${K}_$rep.json'))
print('bake $K', 'c2', round(d['value']*1e6,2), 'us', d['parity'].get('ok'), d.get('launches_per_query'), 'c1', round(e['value']*1e6,2), e['parity'].get('ok'), d.get('bench_s'))"
done
done
