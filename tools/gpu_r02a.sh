# round-2 first evidence: GPU suite, smoke, C3 bench, C5 at N=1 and the N=2 self-launch (gloo, one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_c3_s20.json 2> gpurun_out/bench_c3_s20.err || { tail -30 gpurun_out/bench_c3_s20.err; exit 1; }
cat gpurun_out/bench_c3_s20.json
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > gpurun_out/bench_c5_n1.json 2> gpurun_out/bench_c5_n1.err || { tail -30 gpurun_out/bench_c5_n1.err; exit 1; }
cat gpurun_out/bench_c5_n1.json
timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail -30 gpurun_out/bench_n2.err; exit 1; }
cat gpurun_out/bench_n2.json
timeout -k 10 300 python bench.py --workload c5 --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_c5_n2.json 2> gpurun_out/bench_c5_n2.err || { tail -30 gpurun_out/bench_c5_n2.err; exit 1; }
cat gpurun_out/bench_c5_n2.json
