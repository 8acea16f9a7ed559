set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
LEVELS=1 TOP=0 timeout -k 10 300 python -u tools/program_steps.py c4 4000 > gpurun_out/c4_levels_bytes_4000.txt 2>&1 || { tail -30 gpurun_out/c4_levels_bytes_4000.txt; exit 1; }
LEVELS=1 TOP=0 timeout -k 10 300 python -u tools/program_steps.py c4 1000 > gpurun_out/c4_levels_bytes_1000.txt 2>&1 || { tail -30 gpurun_out/c4_levels_bytes_1000.txt; exit 1; }
grep -- "-- level\|total" gpurun_out/c4_levels_bytes_4000.txt
