# rocprofv3 kernel-trace/stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the C3 bench.
# usage: bash tools/gpu_profile.sh TAG [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r01}; shift
ARGS="$@"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline $ARGS > "$ROOT/gpurun_out/prof_$TAG.json" 2> "$ROOT/gpurun_out/prof_$TAG.err" \
  || { echo "trace pass failed"; tail -20 "$ROOT/gpurun_out/prof_$TAG.err"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$ROOT/gpurun_out/pmc_fetch_$TAG" -o pmc --output-format csv -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline $ARGS > /dev/null 2> "$ROOT/gpurun_out/pmc_fetch_$TAG.err" \
  || { echo "fetch pass failed"; tail -20 "$ROOT/gpurun_out/pmc_fetch_$TAG.err"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$ROOT/gpurun_out/pmc_write_$TAG" -o pmc --output-format csv -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline $ARGS > /dev/null 2> "$ROOT/gpurun_out/pmc_write_$TAG.err" \
  || { echo "write pass failed"; tail -20 "$ROOT/gpurun_out/pmc_write_$TAG.err"; exit 1; }
find "$ROOT/gpurun_out" -name "*stats*.csv" -newer "$ROOT/bench.py" | head
echo done
