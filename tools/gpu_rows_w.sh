# sweep the affine row kernel's row waves per workgroup (PGM_ROWS_W) and store kind
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for W in 1 2 3 4; do
  echo "== W=$W"
  PGM_ROWS_W=$W timeout -k 10 120 python tools/rows_sweep.py --rows 100000 1000000 4000000 --variants lds_values plain_store map_only > gpurun_out/rows_w$W.txt 2>&1 || { tail gpurun_out/rows_w$W.txt; exit 1; }
  cat gpurun_out/rows_w$W.txt
done
for W in 2 4; do
  PGM_ROWS_W=$W timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_w$W.log 2>&1 || { echo "tests W=$W failed"; tail -30 gpurun_out/pytest_w$W.log; exit 1; }
  tail -2 gpurun_out/pytest_w$W.log
done
