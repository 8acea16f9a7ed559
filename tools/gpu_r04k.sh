# round 4: C3 at the driver's 20 steps over the 96 resident batches — user-mode queue count (4 / 6 / 8) and
# the resident ring (started inside the window / resident before it), interleaved, two repeats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04k}
c3() {  # label args...
  local L=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-ring-roofline "$@" > gpurun_out/${TAG}_c3_${L}_$R.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_${L}_$R.json')); r=d['roofline']; print('c3 $L', round(d['value']/1e9,2), 'G frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), d['parity']['ok'])"
}
for R in 1 2; do
  c3 q4 --queues 4
  c3 q6 --queues 6
  c3 q8 --queues 8
  c3 ring --launch ring
  c3 ringpre --launch ring --ring-prestart
done
