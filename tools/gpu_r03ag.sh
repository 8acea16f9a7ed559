# round 3: C4 specialised-step thresholds re-swept after the schedule changes (PGM_PM_JIT_MIN / PGM_PM_PREFER_MIN)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03ag}
for R in 1 2; do
for T in 262144 65536 16384; do
for ROWS in 1000 4000; do
PGM_PM_JIT_MIN=$T PGM_PM_PREFER_MIN=$T timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_t${T}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_t${T}_$R.json')); print('c4 rows $ROWS thresholds $T', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
done
done
