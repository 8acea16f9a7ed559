# round 4: C4 knob sweep at the r04 defaults (merging of a level's specialised steps, write-through / non-
# temporal stores, unroll, rows per lane), 4,000 and 1,000 rows, two interleaved repeats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04v}
c4() {  # label rows env
  local L=$1 ROWS=$2 E=$3
  env $E timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json')); print('c4 $ROWS $L', round(d['value']), round(d['ms_per_step'],3), 'ms')"
}
for R in 1 2; do
  for ROWS in 4000 1000; do
    c4 default $ROWS PGM_NOTHING=1
    c4 merge0 $ROWS PGM_PM_MERGE=0
    c4 wt1 $ROWS PGM_PM_WT=1
    c4 nt0 $ROWS PGM_PM_NT=0
    c4 unroll4 $ROWS PGM_PM_UNROLL=4
    c4 unroll16 $ROWS PGM_PM_UNROLL=16
    c4 xi1 $ROWS PGM_PM_XI=1
    c4 xi4 $ROWS PGM_PM_XI=4
  done
done
