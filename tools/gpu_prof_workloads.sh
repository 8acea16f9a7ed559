# kernel-trace stats of the secondary workloads (C2 single munin query, C4 pathfinder batched BP)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"; TAG=${1:-w}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_${TAG}_c2" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c2 --steps 3 --warmup 1 > "$ROOT/gpurun_out/prof_${TAG}_c2.json" 2> "$ROOT/gpurun_out/prof_${TAG}_c2.err" || { tail -20 "$ROOT/gpurun_out/prof_${TAG}_c2.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_${TAG}_c4" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c4 --rows 1000 --steps 3 --warmup 1 > "$ROOT/gpurun_out/prof_${TAG}_c4.json" 2> "$ROOT/gpurun_out/prof_${TAG}_c4.err" || { tail -20 "$ROOT/gpurun_out/prof_${TAG}_c4.err"; exit 1; }
cat "$ROOT/gpurun_out/prof_${TAG}_c2.json" "$ROOT/gpurun_out/prof_${TAG}_c4.json"
for w in c2 c4; do echo "== $w"; cut -d, -f1-4 "$ROOT/gpurun_out/prof_${TAG}_$w/trace_kernel_stats.csv" | head -8; done
