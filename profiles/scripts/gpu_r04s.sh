# round 4: C4 per-step times at 1,000 and 4,000 rows (each step replayed alone; levels listed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04s}
for ROWS in 1000 4000; do
  LEVELS=1 TOP=40 timeout -k 10 300 python tools/program_steps.py c4 $ROWS > gpurun_out/${TAG}_c4_steps_$ROWS.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c4_steps_$ROWS.txt; exit 1; }
  grep "steps,\|levels:" gpurun_out/${TAG}_c4_steps_$ROWS.txt
done
