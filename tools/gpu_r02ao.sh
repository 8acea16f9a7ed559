set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/floor_bin 100000 > gpurun_out/floor_wt.txt 2>&1 || { tail -20 gpurun_out/floor_wt.txt; exit 1; }
head -12 gpurun_out/floor_wt.txt
