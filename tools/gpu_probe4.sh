# default fused kernel (j-outer, hoisted j-invariant operands) + pair-mode batched products: parity, probe, C4
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p4.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_p4.log; exit 1; }
tail -1 gpurun_out/pytest_p4.log
for R in 1000 4000; do
  for JX in -1 0; do
    PGM_MARG_JX=$JX timeout -k 10 120 python tools/prodn_probe.py $R > gpurun_out/probe4_${R}_$JX.txt 2>&1 || { tail -20 gpurun_out/probe4_${R}_$JX.txt; exit 1; }
    echo "R=$R JX=$JX"; grep fused gpurun_out/probe4_${R}_$JX.txt
  done
  for V in def nopairs; do
    ENVS=""; [ $V = nopairs ] && ENVS="PGM_MARG_JX=0"
    env $ENVS timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/c4p4_${R}_$V.json 2> gpurun_out/c4p4.err || { tail gpurun_out/c4p4.err; exit 1; }
    echo "C4 R=$R $V $(python -c "import json; d=json.load(open('gpurun_out/c4p4_${R}_$V.json')); print(round(d['value']), round(d['ms_per_step'],3), round(d['achieved_GBps']))")"
  done
done
timeout -k 10 120 python tools/program_steps.py c4 4000 > gpurun_out/steps_c4p4_4000.txt 2>&1; head -24 gpurun_out/steps_c4p4_4000.txt | cut -c1-160
