# FP64 GEMM: pgm_gemm vs generic vs vendor (torch.bmm -> rocBLAS, ceiling reference)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm_bench2.txt 2>&1 || { tail -20 gpurun_out/gemm_bench2.txt; exit 1; }
python -c "
import json
for l in open('gpurun_out/gemm_bench2.txt'):
    if l.startswith('{'):
        d=json.loads(l); print(d['batch'],d['M'],d['N'],d['K'],'gemm',round(d['gemm_TFLOPs'],1),'rocblas',round(d['rocblas_ref_TFLOPs'],1),'generic',round(d['generic_TFLOPs'],1))
"
