# r06r: C2 / C1 against the reduction walks' unroll (PGM_CS_UNROLL_PROD for pair jobs, PGM_NARY_UNROLL_PROD
# for n-ary jobs) and workgroups per reducing job (PGM_BATCH_MAX_BLOCKS)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06r; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in 256,16,64 256,64,64 1024,64,64 256,256,64 1024,256,64 256,64,256 1024,64,256; do
  IFS=, read B U N <<< "$cfg"
  export PGM_BATCH_MAX_BLOCKS=$B PGM_CS_UNROLL_PROD=$U PGM_NARY_UNROLL_PROD=$N
  timeout -k 10 200 python bench.py --workload c2 --steps 400 --warmup 40 --no-cpu-baseline > $O/c2_${cfg}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  timeout -k 10 200 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1_${cfg}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/c2_${cfg}_$rep.json')); e=json.load(open('$O/c1_${cfg}_$rep.json'))
print('$cfg', 'c2', round(d['value']*1e6,2), 'us', d['parity'].get('ok'), d.get('launches_per_query'), 'c1', round(e['value']*1e6,2), e['parity'].get('ok'))"
done
done
export PGM_BATCH_MAX_BLOCKS=1024 PGM_CS_UNROLL_PROD=64
timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels.txt 2> $O/levels.err || { tail -30 $O/levels.err; exit 1; }
grep -v "^  level" $O/levels.txt | head -20
