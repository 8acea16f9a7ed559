# round 3: ring waiting backoff A/B (PGM_RING_BACKOFF) at 20 and 400 steps; C2 per-query kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03u}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_plan_gpu.py -k "ring" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 1 2; do
for B in 1 0; do
for S in 20 400; do
PGM_RING_BACKOFF=$B timeout -k 10 300 python bench.py --steps $S --warmup 5 --no-cpu-baseline --no-api-e2e --launch ring --ring-prestart > gpurun_out/${TAG}_rr${S}_b${B}_$R.json 2> gpurun_out/${TAG}_d.err || { tail -30 gpurun_out/${TAG}_d.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_rr${S}_b${B}_$R.json')); r=d['roofline']; print('ringready $S backoff $B', round(d['value']/1e9,2), round(r['frac_wall'],3), d['parity']['ok'])"
done
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c2prof -o c2 --output-format csv -- python3 bench.py --workload c2 --steps 40 --warmup 5 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
F=$(ls gpurun_out/${TAG}_c2prof/*/c2_kernel_trace.csv 2>/dev/null || ls gpurun_out/${TAG}_c2prof/c2_kernel_trace.csv)
python3 tools/c2_trace.py $F 20 25 > gpurun_out/${TAG}_c2_trace.json && head -c 3000 gpurun_out/${TAG}_c2_trace.json
