set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
export PGM_KERNEL_CACHE=$GRAFT_REPO_ROOT/gpurun_out/kc_tmp
$T 300 python -u tools/pm_build_time.py 4000 2>&1 | grep rows
PGM_RTC_THREADS=1 PGM_KERNEL_CACHE=$GRAFT_REPO_ROOT/gpurun_out/kc_tmp1 $T 300 python -u tools/pm_build_time.py 4000 2>&1 | grep rows
$T 300 python -u tools/pm_build_time.py 4000 2>&1 | grep rows
PGM_PM_PREFER_MIN=262144 PGM_KERNEL_CACHE=$GRAFT_REPO_ROOT/gpurun_out/kc_tmp2 $T 300 python -u tools/pm_build_time.py 4000 2>&1 | grep rows
rm -rf gpurun_out/kc_tmp gpurun_out/kc_tmp1 gpurun_out/kc_tmp2
unset PGM_KERNEL_CACHE
$T 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -k "product_n or bp or pathfinder or jt3 or disk_cache or max" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_pm.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_pm.log; exit 1; }
tail -1 gpurun_out/pytest_pm.log
