# r06aa: n-ary fusion budgets re-swept after the 64-entry unroll of pair walks (r06q), with the n-ary nested-loop
# unroll at 64 (default) and 256 (PGM_NARY_UNROLL_PROD)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06aa; mkdir -p $O
export TMPDIR=/tmp
for U in 64 256; do
  PGM_NARY_UNROLL_PROD=$U timeout -k 10 500 python tools/fuse_sweep.py 65536:64 65536:128 65536:256 262144:128 262144:256 1048576:256 65536:64 > $O/sweep_$U.txt 2> $O/sweep_$U.err || { tail -20 $O/sweep_$U.err; exit 1; }
  echo "nary unroll $U"; cat $O/sweep_$U.txt
done
