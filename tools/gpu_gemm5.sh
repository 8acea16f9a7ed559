# FP64 GEMM double-buffered LDS k tiles vs single buffer (PGM_GEMM_SINGLE_BUF): parity, rates, C2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_g4.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_g4.log; exit 1; }
tail -1 gpurun_out/pytest_g4.log
for V in def sbuf; do
  ENVS=""; [ $V = sbuf ] && ENVS="PGM_GEMM_SINGLE_BUF=1"
  env $ENVS timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm_bench5_$V.txt 2>&1 || { tail -20 gpurun_out/gemm_bench5_$V.txt; exit 1; }
  echo "== $V"
  python -c "
import json
for l in open('gpurun_out/gemm_bench5_$V.txt'):
    if l.startswith('{'):
        d=json.loads(l); print(d['batch'],d['M'],d['N'],d['K'],'km/kn',round(d['gemm_TFLOPs'],1),'mk/nk',round(d['gemm_mk_nk_TFLOPs'],1),'rocblas',round(d['rocblas_ref_TFLOPs'],1), 'err', d['max_rel_diff'], d['mk_nk_max_rel_diff'])
"
  env $ENVS timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 2 > gpurun_out/bench_c2_5$V.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_c2_5$V.json')); print('C2 $V', d['value'], d['achieved'])"
done
timeout -k 10 200 python tools/program_steps.py c2 > gpurun_out/steps_c2.txt 2>&1; grep gemm gpurun_out/steps_c2.txt | head -8 | cut -c1-120
