# round 3: C3 release-mode A/B on one box (interleaved), C2/C1 with the host-path changes, C2 profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03p}
for R in 1 2 3 4; do
for M in launch barrier; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --release-mode $M > gpurun_out/${TAG}_direct20_${M}_$R.json 2> gpurun_out/${TAG}_direct20.err || { tail -30 gpurun_out/${TAG}_direct20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_direct20_${M}_$R.json')); r=d['roofline']; print('$M', round(d['value']/1e9,2), round(r['frac'],3), round(r['frac_wall'],3))"
done
done
timeout -k 10 300 python bench.py --workload c1 --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_c1.json 2> gpurun_out/${TAG}_bench_c1.err || { tail -30 gpurun_out/${TAG}_bench_c1.err; exit 1; }
timeout -k 10 300 python bench.py --workload c2 --steps 20 --warmup 2 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { tail -30 gpurun_out/${TAG}_bench_c2.err; exit 1; }
head -c 250 gpurun_out/${TAG}_bench_c1.json gpurun_out/${TAG}_bench_c2.json; echo
timeout -k 10 300 python tools/c2_profile.py > gpurun_out/${TAG}_c2_profile.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c2_profile.txt; exit 1; }
head -30 gpurun_out/${TAG}_c2_profile.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_inference_gpu.py -k "alarm or bn6 or repeated or munin_c2" > gpurun_out/${TAG}_pytest_q.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_q.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_q.log
