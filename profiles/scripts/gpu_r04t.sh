# round 4: C2 per-level kernel trace with the blocks-per-batch-job cap at 256 (default) / 1,024 / 4,096
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04t}
cd /tmp && export TMPDIR=/tmp
for B in 256 1024 4096; do
  PGM_BATCH_MAX_BLOCKS=$B timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/${TAG}_c2trace_$B" -o t --output-format csv -- \
    python3 "$ROOT/tools/c2_level_trace.py" run 200 > "$ROOT/gpurun_out/${TAG}_c2trace_$B.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/${TAG}_c2trace_$B.log"; exit 1; }
done
cd "$ROOT"
for B in 256 1024 4096; do
  python3 tools/c2_level_trace.py summarize gpurun_out/${TAG}_c2trace_$B > gpurun_out/${TAG}_c2_levels_$B.txt
done
paste gpurun_out/${TAG}_c2_levels_256.txt gpurun_out/${TAG}_c2_levels_1024.txt gpurun_out/${TAG}_c2_levels_4096.txt | cut -c1-200
