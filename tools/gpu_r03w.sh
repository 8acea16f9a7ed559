# round 3: C2 with larger contractions joining the level batches (fewer dispatches per level)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03w}
for R in 1 2; do
for MW in 4194304 67108864 1073741824; do
for SW in 65536 4194304 1073741824; do
PGM_BATCH_MAX_WORK=$MW PGM_BATCH_SPLIT_WORK=$SW timeout -k 10 120 python3 bench.py --workload c2 --steps 300 --warmup 20 > gpurun_out/${TAG}_c2_${MW}_${SW}_$R.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_${MW}_${SW}_$R.json')); print('$MW $SW', round(d['value']*1e3,4), 'ms', d['plan'].get('levels'), d['result'][:2])"
done
done
done
PGM_BATCH_MAX_WORK=1073741824 PGM_BATCH_SPLIT_WORK=1073741824 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c2prof -o c2 --output-format csv -- python3 bench.py --workload c2 --steps 40 --warmup 5 > gpurun_out/${TAG}_c2t.json 2> gpurun_out/${TAG}_c2t.err || { tail -30 gpurun_out/${TAG}_c2t.err; exit 1; }
python3 tools/c2_trace.py gpurun_out/${TAG}_c2prof/c2_kernel_trace.csv 20 25 > gpurun_out/${TAG}_c2_trace.json && head -c 1500 gpurun_out/${TAG}_c2_trace.json
