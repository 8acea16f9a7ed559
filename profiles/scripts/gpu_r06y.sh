# r06y: the direct-chain tests, including the split last level
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "direct_chain" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest.log | tail -5
