# kernel-trace of one bench invocation: bash tools/gpu_trace.sh TAG bench-args...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"; TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/tr_$TAG" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" "$@" > "$ROOT/gpurun_out/tr_$TAG.json" 2> "$ROOT/gpurun_out/tr_$TAG.err" || { tail -20 "$ROOT/gpurun_out/tr_$TAG.err"; exit 1; }
cat "$ROOT/gpurun_out/tr_$TAG.json"
python3 "$ROOT/tools/trace_summary.py" "$ROOT/gpurun_out/tr_$TAG/trace_kernel_trace.csv"
