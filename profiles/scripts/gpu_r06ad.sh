# r06ad: fusion budgets around 256 Ki / 512 with the split n-ary walks (two passes)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ad; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 500 python tools/fuse_sweep.py 65536:64 131072:256 131072:512 262144:512 262144:1024 524288:512 524288:1024 > $O/sweep_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep_$rep.txt
done
