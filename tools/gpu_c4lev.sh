# levelled batched BP: parity, then C4 bench at 1000/4000 rows (levelled vs per-step, batch-size knob)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_c4.log; exit 1; }
tail -2 gpurun_out/pytest_c4.log
for R in 1000 4000; do
  for V in "lev" "seq" "b16" "b21"; do
    case $V in
      lev) ENVS="";;
      seq) ENVS="PGM_BP_LEVELS=0";;
      b16) ENVS="PGM_PRODN_BATCH_MAX=65536";;
      b21) ENVS="PGM_PRODN_BATCH_MAX=2097152";;
    esac
    env $ENVS timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/bench_c4_${R}_$V.json 2> gpurun_out/bench_c4_${R}_$V.err || { tail gpurun_out/bench_c4_${R}_$V.err; exit 1; }
    echo "$R $V $(cat gpurun_out/bench_c4_${R}_$V.json)"
  done
done
timeout -k 10 120 python tools/program_steps.py c4 1000 > gpurun_out/steps_c4lev_1000.txt 2>&1; head -30 gpurun_out/steps_c4lev_1000.txt | cut -c1-200
