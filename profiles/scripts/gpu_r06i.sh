# r06i: n-ary fusion settings swept on C2 / C1 (chain time and query time)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python tools/fuse_sweep.py 0:0 16384:64:0 16384:64:1 65536:64:1 65536:128:1 65536:256:1 262144:128:1 16384:16:1 32768:32:1 0:0 > $O/sweep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.txt
