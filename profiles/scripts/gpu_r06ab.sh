# r06ab: n-ary jobs whose G lanes stride over the outer reduction dims only, the inner dims as literal loops
# (PGM_NARY_SPLIT=1) against the flattened per-entry decode (0): the n-ary tests, then fusion budgets on C2 / C1
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "contract_n or fused_query" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for S in 1 0; do
  PGM_NARY_SPLIT=$S timeout -k 10 500 python tools/fuse_sweep.py 65536:64 65536:256 262144:256 262144:512 1048576:512 > $O/sweep_$S.txt 2> $O/sweep_$S.err || { tail -20 $O/sweep_$S.err; exit 1; }
  echo "split $S"; cat $O/sweep_$S.txt
done
