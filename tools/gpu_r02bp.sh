# k_gemm_f64: running k offsets on the 64x64 tile only; GEMM tests + A/B vs the HEAD kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/bp_pytest.log 2>&1 || { tail -30 gpurun_out/bp_pytest.log; exit 1; }
tail -1 gpurun_out/bp_pytest.log
for v in old cur old cur; do
  L=pgmpy_amd/lib/libpgmhip_$v.so; [ $v = cur ] && L=pgmpy_amd/lib/libpgmhip.so
  PGM_LIB_PATH=$PWD/$L timeout -k 10 300 python3 tools/gemm_bench.py > gpurun_out/bp_$v.txt 2>&1 || { tail -20 gpurun_out/bp_$v.txt; exit 1; }
  python3 -c "
import json,sys
out=[]
for l in open('gpurun_out/bp_$v.txt'):
    if l.startswith('{'):
        d=json.loads(l); out.append(f\"{d['batch']}x{d['M']}x{d['N']}x{d['K']}:{d['gemm_us']:.0f}us/{d['gemm_TFLOPs']:.1f}TF\")
print('$v', ' '.join(out))"
done
