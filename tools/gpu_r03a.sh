# round 3, first GPU pass: Markov-network tests, the resident ring kernel (parity + exits), RCCL at
# world 1, then C3 through the ring vs the 4-queue direct dispatch, and a rocprofv3 kernel trace of
# the ring bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03a}
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_plan_gpu.py -k "ring" > gpurun_out/${TAG}_pytest_ring.log 2>&1 || { echo ring tests failed; tail -60 gpurun_out/${TAG}_pytest_ring.log; exit 1; }
tail -4 gpurun_out/${TAG}_pytest_ring.log
timeout -k 10 300 $T -m gpu tests/test_markov.py > gpurun_out/${TAG}_pytest_markov.log 2>&1 || { echo markov tests failed; tail -60 gpurun_out/${TAG}_pytest_markov.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_markov.log
timeout -k 10 400 $T -m gpu tests/test_distributed.py > gpurun_out/${TAG}_pytest_dist.log 2>&1 || { echo dist tests failed; tail -60 gpurun_out/${TAG}_pytest_dist.log; exit 1; }
tail -4 gpurun_out/${TAG}_pytest_dist.log
timeout -k 10 300 python bench.py --launch ring --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_ring20.json 2> gpurun_out/${TAG}_bench_ring20.err || { tail -30 gpurun_out/${TAG}_bench_ring20.err; exit 1; }
timeout -k 10 300 python bench.py --launch ring --steps 400 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_ring400.json 2> gpurun_out/${TAG}_bench_ring400.err || { tail -30 gpurun_out/${TAG}_bench_ring400.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_direct20.json 2> gpurun_out/${TAG}_bench_direct20.err || { tail -30 gpurun_out/${TAG}_bench_direct20.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_ring -o ring -- python3 bench.py --launch ring --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_ring20_prof.json 2> gpurun_out/${TAG}_bench_ring20_prof.err || { tail -30 gpurun_out/${TAG}_bench_ring20_prof.err; exit 1; }
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d.get("roofline") or {}
    print(f, {k: d.get(k) for k in ("value","ms_per_step")}, {k: r.get(k) for k in ("frac","frac_wall","kernel","kernel_ms","grid","single_launch_kernel_ms")}, (d.get("parity") or {}).get("ok"))'
python -c "$P" gpurun_out/${TAG}_bench_*.json
