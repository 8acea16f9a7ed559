# round 4: run-to-run spread on one box at HEAD — the driver's C3 line five times, C2 / C4 three times each
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04y}
for R in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_c3_$R.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_$R.json')); r=d['roofline']; print('c3', round(d['value']/1e9,2), 'G frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), 'ring', round(r['single_launch_ring']['frac'],3))"
done
for R in 1 2 3; do
  timeout -k 10 300 python bench.py --workload c2 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_c2_$R.json 2> gpurun_out/${TAG}_c2.err || { tail -20 gpurun_out/${TAG}_c2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_$R.json')); print('c2', round(d['value']*1e3,4), 'ms')"
  for ROWS in 4000 1000; do
    timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_c4_${ROWS}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -20 gpurun_out/${TAG}_c4.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_$R.json')); print('c4 $ROWS', round(d['value']), round(d['ms_per_step'],3), 'ms')"
  done
done
