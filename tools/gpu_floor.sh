set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 60 ./tools/floor 100000 > gpurun_out/floor_100k.txt 2>&1 && cat gpurun_out/floor_100k.txt
timeout -k 10 120 python tools/rows_sweep.py --rows 100000 1000000 --variants lds_values compact_codes global_values > gpurun_out/rows_compact.txt 2>&1; cat gpurun_out/rows_compact.txt
