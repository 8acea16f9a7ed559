# round 3: ring posts by direct counter stores (absolute counter, no per-launch reset), compiled classic VE
# and BP out-of-clique queries; full GPU suite, ring vs direct C3, rocprof of the ring line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03e}
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_plan_gpu.py -k "ring" > gpurun_out/${TAG}_pytest_ring.log 2>&1 || { echo ring tests failed; tail -60 gpurun_out/${TAG}_pytest_ring.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_ring.log
timeout -k 10 600 $T -m gpu tests/test_inference_gpu.py tests/test_markov.py > gpurun_out/${TAG}_pytest_inf.log 2>&1 || { echo inference tests failed; tail -80 gpurun_out/${TAG}_pytest_inf.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_inf.log
for K in 20 100 400; do
timeout -k 10 300 python bench.py --launch ring --steps $K --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_ring$K.json 2> gpurun_out/${TAG}_bench_ring$K.err || { tail -30 gpurun_out/${TAG}_bench_ring$K.err; exit 1; }
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_direct20.json 2> gpurun_out/${TAG}_bench_direct20.err || { tail -30 gpurun_out/${TAG}_bench_direct20.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_ring -o ring -- python3 bench.py --launch ring --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_ring20_prof.json 2> gpurun_out/${TAG}_bench_ring20_prof.err || { tail -30 gpurun_out/${TAG}_bench_ring20_prof.err; exit 1; }
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d.get("roofline") or {}
    print(f, {k: d.get(k) for k in ("value","ms_per_step")}, {k: r.get(k) for k in ("frac","frac_wall","kernel","kernel_ms","kernel_span_ms","single_launch_kernel_ms")}, (d.get("parity") or {}).get("ok"))'
python -c "$P" gpurun_out/${TAG}_bench_*.json
find gpurun_out/${TAG}_prof_ring -name "*kernel_stats.csv" -exec head -4 {} \;
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
LEVELS=1 TOP=10 timeout -k 10 300 python tools/program_steps.py c4 4000 > gpurun_out/${TAG}_c4_levels.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c4_levels.txt; exit 1; }
LEVELS=1 TOP=10 timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_levels.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c2_levels.txt; exit 1; }
head -3 gpurun_out/${TAG}_c4_levels.txt gpurun_out/${TAG}_c2_levels.txt
