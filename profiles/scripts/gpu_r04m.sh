# round 4: where C2's 0.18 ms go — a kernel trace of 200 complete queries (per-level kernel time and the gap
# before each launch), plus the same for C1 (alarm)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04m}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/${TAG}_c2trace" -o t --output-format csv -- \
  python3 "$ROOT/tools/c2_level_trace.py" run 200 > "$ROOT/gpurun_out/${TAG}_c2trace.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/${TAG}_c2trace.log"; exit 1; }
cd "$ROOT"
grep "queries" gpurun_out/${TAG}_c2trace.log
python3 tools/c2_level_trace.py summarize gpurun_out/${TAG}_c2trace > gpurun_out/${TAG}_c2_levels.txt && cat gpurun_out/${TAG}_c2_levels.txt
timeout -k 10 300 python3 tools/c2_level_trace.py run 200 > gpurun_out/${TAG}_c2_noprof.log 2>&1 && cat gpurun_out/${TAG}_c2_noprof.log | grep queries
