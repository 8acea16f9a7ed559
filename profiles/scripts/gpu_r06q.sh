# r06q: C2 / C1 against the batch jobs' lanes-per-output cap, workgroups per job and the reduction
# walk's unroll (A/B knobs PGM_BATCH_LANES_CAP, PGM_BATCH_MAX_BLOCKS, PGM_BATCH_MAX_BLOCKS_PRODUCT,
# PGM_CS_UNROLL_PROD)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06q; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in 4096,256,1024,16 16384,256,1024,16 4096,1024,1024,16 16384,1024,4096,16 4096,256,1024,64 16384,1024,1024,64 65536,1024,1024,16; do
  IFS=, read L B P U <<< "$cfg"
  export PGM_BATCH_LANES_CAP=$L PGM_BATCH_MAX_BLOCKS=$B PGM_BATCH_MAX_BLOCKS_PRODUCT=$P PGM_CS_UNROLL_PROD=$U
  timeout -k 10 200 python bench.py --workload c2 --steps 400 --warmup 40 --no-cpu-baseline > $O/c2_${cfg}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  timeout -k 10 200 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1_${cfg}_$rep.json 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/c2_${cfg}_$rep.json')); e=json.load(open('$O/c1_${cfg}_$rep.json'))
print('$cfg', 'c2', round(d['value']*1e6,2), 'us', d['parity'].get('ok'), d.get('launches_per_query'), 'c1', round(e['value']*1e6,2), e['parity'].get('ok'))"
done
done
unset PGM_BATCH_LANES_CAP PGM_BATCH_MAX_BLOCKS PGM_BATCH_MAX_BLOCKS_PRODUCT PGM_CS_UNROLL_PROD
