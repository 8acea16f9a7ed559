# r06o: C2 (and C1) chain with the inner packets' fences at agent scope (default) or none (timing A/B only:
# without them a step may read stale lines, the parity field says whether it did)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp
for AR in 11 01 10 00 11 01 10 00; do
  A=${AR:0:1}; R=${AR:1:1}
  PGM_DQ_CHAIN_ACQ=$A PGM_DQ_CHAIN_REL=$R timeout -k 10 200 python bench.py --workload c2 --steps 400 --warmup 40 --no-cpu-baseline > $O/c2_$AR.json 2>> $O/c2.err \
    || { tail -30 $O/c2.err; exit 1; }
  PGM_DQ_CHAIN_ACQ=$A PGM_DQ_CHAIN_REL=$R timeout -k 10 200 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1_$AR.json 2>> $O/c2.err \
    || { tail -30 $O/c2.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/c2_$AR.json')); e=json.load(open('$O/c1_$AR.json'))
print('acq $A rel $R', 'c2', round(d['value']*1e6,2), 'us', d['parity'].get('ok'), d['parity'].get('max_abs_err'), (d.get('roofline') or {}).get('chain_us'), 'c1', round(e['value']*1e6,2), e['parity'].get('ok'))"
done
