# r06ak: n-ary jobs' G lanes of an output at stride 64/G within a wave (PGM_NARY_LANEMAP=1) against adjacent (0):
# the n-ary tests, then C2 / C1 (two passes each)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ak; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "contract_n or fused_query or munin_c2 or alarm" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for LM in 1 0; do
  PGM_NARY_LANEMAP=$LM timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_${LM}_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  echo "lanemap $LM"; cat $O/sweep_${LM}_$rep.txt
done
done
PGM_NARY_LANEMAP=1 FUSED_ONLY=1 timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels.txt
