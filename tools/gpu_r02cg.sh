# round-2 closing evidence (rocprof + PMC already in r02cf): GPU suite incl. the full-belief C4 test, smoke, C3 20 steps, C5 N=1, C1, e2e
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02cg}
timeout -k 10 240 python -u -m pytest tests/test_inference_gpu.py -k full_beliefs -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_c4full.log 2>&1 || { echo c4 full failed; tail -40 gpurun_out/pytest_c4full.log; exit 1; }
tail -3 gpurun_out/pytest_c4full.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || { tail -30 gpurun_out/${TAG}_bench_c3.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.err || { tail -30 gpurun_out/${TAG}_bench_c5.err; exit 1; }
timeout -k 10 300 python bench.py --workload c1 --steps 100 --warmup 2 > gpurun_out/${TAG}_bench_c1.json 2> gpurun_out/${TAG}_bench_c1.err || { tail -30 gpurun_out/${TAG}_bench_c1.err; exit 1; }
timeout -k 10 300 python tools/e2e_predict.py 100000 > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -30 gpurun_out/${TAG}_e2e.err; exit 1; }
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); print(f, {k: d.get(k) for k in ("value","unit","ms_per_step")}, (d.get("roofline") or {}).get("frac"))'
python -c "$P" gpurun_out/${TAG}_bench_*.json
