# r05o: per-step C4 dump at HEAD (4,000 and 1,000 rows)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05o
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c4_dump.py gpurun_out/r05o/d4000 > gpurun_out/r05o/d4000.log 2>&1 || { tail -20 gpurun_out/r05o/d4000.log; exit 1; }
ROWS=1000 timeout -k 10 300 python -u tools/c4_dump.py gpurun_out/r05o/d1000 > gpurun_out/r05o/d1000.log 2>&1 || { tail -20 gpurun_out/r05o/d1000.log; exit 1; }
cat gpurun_out/r05o/d4000.log gpurun_out/r05o/d1000.log
