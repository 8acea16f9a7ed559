set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --steps 400 --warmup 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo bench failed; tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo c2 failed; tail -30 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 300 python bench.py --workload c4 --rows 1000 --steps 5 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo c4 failed; tail -30 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
