set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; ROOT=$GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/floor 100000 > gpurun_out/floor_100k.txt 2>&1 && cat gpurun_out/floor_100k.txt
timeout -k 10 60 ./tools/floor 1000000 > gpurun_out/floor_1m.txt 2>&1 && cat gpurun_out/floor_1m.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_floor -o trace --output-format csv -- $ROOT/tools/floor 100000 > /dev/null 2>&1 || exit 1
cut -d, -f1-6 $ROOT/gpurun_out/prof_floor/trace_kernel_stats.csv
cd $ROOT && bash tools/gpu_profile.sh r01e --steps 50 --warmup 5
