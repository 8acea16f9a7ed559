# diagnose: random-pattern steps path with the stale-error probe, then the thread test
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
PGM_STALE_PROBE=1 timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -k "random_patterns" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_rp.log 2>&1; echo rc=$?
grep -n "pending HIP error" gpurun_out/pytest_rp.log | head -20
tail -5 gpurun_out/pytest_rp.log
timeout -k 10 300 python -u -m pytest tests/test_inference_gpu.py -k "threads or late_edits" -v --timeout 120 --timeout-method thread > gpurun_out/pytest_thr.log 2>&1; echo rc=$?
tail -5 gpurun_out/pytest_thr.log
