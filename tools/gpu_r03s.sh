# round 3: resident ring started ready before the window (pgm_rows_ring_start_ready) vs direct, 20 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03s}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_plan_gpu.py -k "ring or direct" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 1 2 3; do
for M in ringready ring direct; do
case $M in
  ringready) A="--launch ring --ring-prestart";;
  ring) A="--launch ring";;
  direct) A="";;
esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e $A > gpurun_out/${TAG}_${M}20_$R.json 2> gpurun_out/${TAG}_d.err || { tail -30 gpurun_out/${TAG}_d.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_${M}20_$R.json')); r=d['roofline']; print('$M', round(d['value']/1e9,2), round(r['frac'],3), round(r['frac_wall'],3), d['config'].get('ring_host_launch_ms'), d['parity']['ok'])"
done
done
