# r06as: level batches' jobs added heaviest first (PGM_BATCH_SORT=1) vs recording order (0): kernel / inference
# GPU suites with it, C2 / C1 sweep twice, per-launch times with it
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06as; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for BS in 1 0; do
  PGM_BATCH_SORT=$BS timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_${BS}_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  echo "sort $BS"; cat $O/sweep_${BS}_$rep.txt
done
done
FUSED_ONLY=1 timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels.txt
