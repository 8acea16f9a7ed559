# round 3: C4 fused-pass block floor x specialised-step threshold, after r03ag
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03ai}
for R in 1 2; do
for MB in 32 8 2; do
for T in 16384; do
for ROWS in 1000 4000; do
PGM_MARG_MIN_BLOCKS=$MB PGM_PM_JIT_MIN=$T PGM_PM_PREFER_MIN=$T timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_m${MB}_t${T}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_m${MB}_t${T}_$R.json')); print('c4 rows $ROWS min_blocks $MB thresholds $T', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
done
done
done
