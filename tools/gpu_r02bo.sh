# k_gemm_f64 A/B: HEAD kernel (old), strength-reduced offsets with LDS pad 1 (current) and pad 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in old cur p2 old cur p2; do
  L=pgmpy_amd/lib/libpgmhip_$v.so; [ $v = cur ] && L=pgmpy_amd/lib/libpgmhip.so
  PGM_LIB_PATH=$PWD/$L timeout -k 10 300 python3 tools/gemm_bench.py > gpurun_out/bo_$v.txt 2>&1 || { tail -20 gpurun_out/bo_$v.txt; exit 1; }
  python3 -c "
import json,sys
out=[]
for l in open('gpurun_out/bo_$v.txt'):
    if l.startswith('{'):
        d=json.loads(l); out.append(f\"{d['batch']}x{d['M']}x{d['N']}x{d['K']}:{d['gemm_us']:.0f}us/{d['gemm_TFLOPs']:.1f}TF\")
print('$v', ' '.join(out))"
done
