set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for B in 64 128 256 512; do
  PGM_JIT_BLOCK=$B timeout -k 10 120 python tools/rows_sweep.py --rows 100000 1000000 --reps 400 --variants lds_values > gpurun_out/jit_b$B.txt 2>&1; echo "B=$B $(grep -o '"rows": [0-9]*\|"kernel_us": [0-9.]*' gpurun_out/jit_b$B.txt | tr '\n' ' ')"
  PGM_JIT_GLOBAL_VALUES=1 PGM_JIT_BLOCK=$B timeout -k 10 120 python tools/rows_sweep.py --rows 100000 1000000 --reps 400 --variants lds_values > gpurun_out/jit_g$B.txt 2>&1; echo "GLOBAL B=$B $(grep -o '"rows": [0-9]*\|"kernel_us": [0-9.]*' gpurun_out/jit_g$B.txt | tr '\n' ' ')"
done
