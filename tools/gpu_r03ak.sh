# round 3: C4 knobs re-checked after the schedule changes (PGM_PRODN_BATCH_MAX, PGM_PM_XI_MIN, PGM_BP_LAYOUT)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03ak}
run() {  # label env...
  local L=$1; shift
  for ROWS in 1000 4000; do
    env "$@" timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_${L}_$R.json')); print('c4 rows $ROWS $L', round(d['value']), round(d['ms_per_step'],3), 'ms')"
  done
}
for R in 1 2; do
run default PGM_NOTHING=1
run pbm256k PGM_PRODN_BATCH_MAX=262144
run pbm64k PGM_PRODN_BATCH_MAX=65536
run xi1 PGM_PM_XI_MIN=1
run layout1 PGM_BP_LAYOUT=1
done
