# round 3: where C2's per-query GPU time goes (kernel durations vs gaps), from a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03t}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c2prof -o c2 --output-format csv -- python3 bench.py --workload c2 --steps 40 --warmup 5 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
F=$(ls gpurun_out/${TAG}_c2prof/*/c2_kernel_trace.csv 2>/dev/null || ls gpurun_out/${TAG}_c2prof/c2_kernel_trace.csv)
python3 tools/c2_trace.py $F 20 25 > gpurun_out/${TAG}_c2_trace.json && head -c 3000 gpurun_out/${TAG}_c2_trace.json
