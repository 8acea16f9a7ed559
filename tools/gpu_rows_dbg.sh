# strip pieces of the affine row kernel (PGM_ROWS_DBG mask) to locate its per-launch time
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for D in 0 1 2 4 8 12 13 15; do
  echo "== DBG=$D"
  PGM_ROWS_DBG=$D timeout -k 10 120 python tools/rows_sweep.py --rows 100000 --reps 50 --variants lds_values > gpurun_out/rows_dbg$D.txt 2>&1 || { tail gpurun_out/rows_dbg$D.txt; exit 1; }
  grep kernel_us gpurun_out/rows_dbg$D.txt
done
