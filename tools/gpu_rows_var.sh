set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for X in 0 1; do for D in 0 96; do
  if [ $X = 1 ]; then export PGM_ROWS_XFULL=1; else unset PGM_ROWS_XFULL; fi
  PGM_ROWS_DBG=$D timeout -k 10 120 python tools/rows_sweep.py --rows 100000 1000000 4000000 --reps 30 --variants lds_values > gpurun_out/rows_var$D.txt 2>&1 || exit 1
  echo "XFULL=$X DBG=$D $(grep -o '"rows": [0-9]*\|"kernel_us": [0-9.]*' gpurun_out/rows_var$D.txt | tr '\n' ' ')"
done; done
