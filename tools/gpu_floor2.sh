set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; ROOT=$GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/floor 100000 > gpurun_out/floor_100k.txt 2>&1 && cat gpurun_out/floor_100k.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_floor2 -o trace --output-format csv -- $ROOT/tools/floor 100000 > /dev/null 2>&1 || exit 1
cut -d, -f1-4 $ROOT/gpurun_out/prof_floor2/trace_kernel_stats.csv
PGM_ROWS_DBG=15 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_dbg15 -o trace --output-format csv -- python3 $ROOT/tools/rows_sweep.py --rows 100000 --reps 50 --variants lds_values > /dev/null 2>&1 || exit 1
cut -d, -f1-4 $ROOT/gpurun_out/prof_dbg15/trace_kernel_stats.csv
