set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py tests/test_factor_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bpc.log 2>&1 || { echo failed; tail -60 gpurun_out/pytest_bpc.log; exit 1; }
tail -1 gpurun_out/pytest_bpc.log
timeout -k 10 300 python -u tools/c4_single.py > gpurun_out/c4_single.json 2> gpurun_out/c4_single.err || { tail -30 gpurun_out/c4_single.err; exit 1; }
cat gpurun_out/c4_single.json
