# round 3: single-query wait A/B (PGM_SYNC_SPIN) on C1 / C2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03ab}
for R in 1 2; do
for S in 1 0; do
PGM_SYNC_SPIN=$S timeout -k 10 120 python3 bench.py --workload c2 --steps 300 --warmup 20 > gpurun_out/${TAG}_c2_s${S}_$R.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_s${S}_$R.json')); print('c2 spin$S', round(d['value']*1e3,4), 'ms', d['result'][:2])"
PGM_SYNC_SPIN=$S timeout -k 10 300 python3 bench.py --workload c1 --steps 100 --warmup 5 > gpurun_out/${TAG}_c1_s${S}_$R.json 2> gpurun_out/${TAG}_c1.err || { tail -30 gpurun_out/${TAG}_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c1_s${S}_$R.json')); print('c1 spin$S', round(d['value']*1e3,4), 'ms')"
done
done
