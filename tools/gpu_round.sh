# full round evidence: GPU tests, smoke, bench (all workloads), rocprof + PMC of the C3 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_bench.sh || exit 1
bash tools/gpu_profile.sh $TAG --steps 200 --warmup 10 || exit 1
