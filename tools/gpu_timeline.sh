set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PGM_ROWS_DBG=16 timeout -k 10 120 python tools/rows_timeline.py 100000 > gpurun_out/timeline_100k.txt 2>&1; tail -3 gpurun_out/timeline_100k.txt
PGM_ROWS_DBG=16 timeout -k 10 120 python tools/rows_timeline.py 1000000 > gpurun_out/timeline_1m.txt 2>&1; tail -3 gpurun_out/timeline_1m.txt
