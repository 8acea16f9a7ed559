# r05g: C4 merge policy A/B: big specialised steps launched alone (PGM_PM_MERGE_MAX_MB), merged bodies sorted
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05g
export TMPDIR=/tmp
run() {  # label rows env...
  local L=$1 R=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05g/c4_${L}_$R.json 2> gpurun_out/r05g/c4.err || { tail -20 gpurun_out/r05g/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05g/c4_${L}_$R.json')); print('$L', $R, round(d['value']/1e6,4), 'M/s', d['parity']['ok'])"
}
for rep in 1 2; do
for R in 4000 1000; do
  run base $R PGM_NOTHING=1
  run m8 $R PGM_PM_MERGE_MAX_MB=8
  run m32 $R PGM_PM_MERGE_MAX_MB=32
  run m128 $R PGM_PM_MERGE_MAX_MB=128
  run sort $R PGM_PM_MERGE_SORT=1
  run m32sort $R PGM_PM_MERGE_MAX_MB=32 PGM_PM_MERGE_SORT=1
done
done
