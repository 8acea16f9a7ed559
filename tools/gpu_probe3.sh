# fused product+marginal: j-inner (JX=0) vs j-outer (JX=1,2,4) kernels — parity then probe rates, C4 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for JX in 1 2 4; do
  PGM_MARG_JX=$JX timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "marginal or bp" --timeout 120 --timeout-method thread > gpurun_out/pytest_jx$JX.log 2>&1 || { echo "tests failed JX=$JX"; tail -30 gpurun_out/pytest_jx$JX.log; exit 1; }
  echo "JX=$JX $(tail -1 gpurun_out/pytest_jx$JX.log)"
done
for R in 1000 4000; do
  for JX in 0 1 2 4; do
    PGM_MARG_JX=$JX timeout -k 10 120 python tools/prodn_probe.py $R > gpurun_out/probe3_${R}_$JX.txt 2>&1 || { tail -20 gpurun_out/probe3_${R}_$JX.txt; exit 1; }
    echo "R=$R JX=$JX"; grep fused gpurun_out/probe3_${R}_$JX.txt
  done
  for JX in 0 2 4; do
    PGM_MARG_JX=$JX timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/c4jx.json 2> gpurun_out/c4jx.err || { tail gpurun_out/c4jx.err; exit 1; }
    echo "C4 R=$R JX=$JX $(python -c "import json; d=json.load(open('gpurun_out/c4jx.json')); print(round(d['value']), round(d['ms_per_step'],3), round(d['achieved_GBps']))")"
  done
done
