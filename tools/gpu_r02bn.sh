# k_gemm_f64: strength-reduced k offsets + 1-double LDS padding: GEMM tests, gemm_bench, SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/bn_pytest.log 2>&1 || { tail -30 gpurun_out/bn_pytest.log; exit 1; }
tail -1 gpurun_out/bn_pytest.log
timeout -k 10 300 python3 tools/gemm_bench.py > gpurun_out/bn_gemm_bench.txt 2>&1 || { tail -20 gpurun_out/bn_gemm_bench.txt; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/bn_gemm_bench.txt'):
    if l.startswith('{'):
        d=json.loads(l); print(d['batch'],d['M'],d['N'],d['K'],'gemm',round(d['gemm_us'],1),'us',round(d['gemm_TFLOPs'],1),'TF mknk',round(d['gemm_mk_nk_TFLOPs'],1),'rocblas',round(d['rocblas_ref_TFLOPs'],1),'rel',d['max_rel_diff'])"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -d "$ROOT/gpurun_out/bn_pmc_sq" -o pmc --output-format csv -- python3 "$ROOT/tools/gemm_bench.py" > "$ROOT/gpurun_out/bn_pmc_sq.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/bn_pmc_sq.log"; exit 1; }
echo done
