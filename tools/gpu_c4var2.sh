# C4 variants: fused-marginal load batching (PGM_MARG_U) x level-batch size (PGM_PRODN_BATCH_MAX)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 env PGM_MARG_U=4 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "marginal or bp" --timeout 120 --timeout-method thread > gpurun_out/pytest_c4u.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_c4u.log; exit 1; }
tail -1 gpurun_out/pytest_c4u.log
for R in 1000 4000; do
  for V in "u1" "u2" "u4" "u4b22" "u4b23"; do
    case $V in
      u1) ENVS="PGM_MARG_U=1";;
      u2) ENVS="PGM_MARG_U=2";;
      u4) ENVS="PGM_MARG_U=4";;
      u4b22) ENVS="PGM_MARG_U=4 PGM_PRODN_BATCH_MAX=4194304";;
      u4b23) ENVS="PGM_MARG_U=4 PGM_PRODN_BATCH_MAX=8388608";;
    esac
    env $ENVS timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/bench_c4_${R}_$V.json 2> gpurun_out/bench_c4_${R}_$V.err || { tail gpurun_out/bench_c4_${R}_$V.err; exit 1; }
    echo "$R $V $(python -c "import json; d=json.load(open('gpurun_out/bench_c4_${R}_$V.json')); print(round(d['value']), round(d['ms_per_step'],3), round(d['achieved_GBps']))")"
  done
done
PGM_MARG_U=4 timeout -k 10 120 python tools/program_steps.py c4 1000 > gpurun_out/steps_c4u4_1000.txt 2>&1; head -12 gpurun_out/steps_c4u4_1000.txt | cut -c1-160
PGM_MARG_U=4 timeout -k 10 120 python tools/program_steps.py c4 4000 > gpurun_out/steps_c4u4_4000.txt 2>&1; head -16 gpurun_out/steps_c4u4_4000.txt | cut -c1-160
