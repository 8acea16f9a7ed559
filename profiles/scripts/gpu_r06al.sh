# r06al: the 64/G lane stride for pair jobs too: kernel / inference / plan GPU suites, C2 / C1 sweep, C2 per-job times
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06al; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py tests/test_plan_gpu.py tests/test_compat_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  cat $O/sweep_$rep.txt
done
FUSED_ONLY=1 JOB_TIMES=1 timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels_jobs.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels_jobs.txt
