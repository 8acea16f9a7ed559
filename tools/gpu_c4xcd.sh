# XCD-aware block order for the j-outer fused product+marginal kernel (PGM_MARG_XCD): parity, C4 at 1000/4000
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PGM_MARG_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "marginal or bp" --timeout 120 --timeout-method thread > gpurun_out/pytest_xcd.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_xcd.log; exit 1; }
tail -1 gpurun_out/pytest_xcd.log
for R in 1000 4000; do
  for X in 0 1 0 1; do
    PGM_MARG_XCD=$X timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/c4x.json 2> gpurun_out/c4x.err || { tail gpurun_out/c4x.err; exit 1; }
    echo "C4 R=$R XCD=$X $(python -c "import json; d=json.load(open('gpurun_out/c4x.json')); print(round(d['value']), round(d['ms_per_step'],3), round(d['achieved_GBps']))")"
  done
done
PGM_MARG_XCD=1 timeout -k 10 120 python tools/program_steps.py c4 4000 > gpurun_out/steps_c4xcd_4000.txt 2>&1; head -8 gpurun_out/steps_c4xcd_4000.txt | cut -c1-120
