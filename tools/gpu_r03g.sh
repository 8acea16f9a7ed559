# round 3: C1 check (query_one), levelled-chain diagnostic, inference suites, C3 ring vs direct, C4 levels
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03g}
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 python -u tools/c1_check.py --chain > gpurun_out/${TAG}_c1_check.txt 2>&1 || { tail -8 gpurun_out/${TAG}_c1_check.txt; exit 1; }; tail -3 gpurun_out/${TAG}_c1_check.txt
timeout -k 10 300 python bench.py --workload c1 --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_c1.json 2> gpurun_out/${TAG}_bench_c1.err || { tail -30 gpurun_out/${TAG}_bench_c1.err; exit 1; }
timeout -k 10 300 python bench.py --workload c2 --steps 20 --warmup 2 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { tail -30 gpurun_out/${TAG}_bench_c2.err; exit 1; }
head -c 300 gpurun_out/${TAG}_bench_c1.json gpurun_out/${TAG}_bench_c2.json; echo
LEVELS=1 TOP=10 timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_levels.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c2_levels.txt; exit 1; }
head -3 gpurun_out/${TAG}_c2_levels.txt
timeout -k 10 600 $T -m gpu tests/test_inference_gpu.py tests/test_markov.py > gpurun_out/${TAG}_pytest_inf.log 2>&1 || { echo inference tests failed; tail -80 gpurun_out/${TAG}_pytest_inf.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_inf.log
for K in 20 400; do
timeout -k 10 300 python bench.py --launch ring --steps $K --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_ring$K.json 2> gpurun_out/${TAG}_bench_ring$K.err || { tail -30 gpurun_out/${TAG}_bench_ring$K.err; exit 1; }
timeout -k 10 300 python bench.py --steps $K --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_direct$K.json 2> gpurun_out/${TAG}_bench_direct$K.err || { tail -30 gpurun_out/${TAG}_bench_direct$K.err; exit 1; }
done
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d.get("roofline") or {}
    print(f, {k: d.get(k) for k in ("value","ms_per_step")}, {k: r.get(k) for k in ("frac","frac_wall","kernel","kernel_ms","single_launch_kernel_ms","single_queue_kernel_ms")}, (d.get("parity") or {}).get("ok"))'
python -c "$P" gpurun_out/${TAG}_bench_ring*.json gpurun_out/${TAG}_bench_direct*.json
LEVELS=1 TOP=10 timeout -k 10 300 python tools/program_steps.py c4 4000 > gpurun_out/${TAG}_c4_levels.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c4_levels.txt; exit 1; }
head -3 gpurun_out/${TAG}_c4_levels.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
