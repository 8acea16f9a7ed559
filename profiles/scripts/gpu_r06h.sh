# r06h: n-ary fusion settings swept on C2 / C1 (chain time and query time)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python tools/fuse_sweep.py 0:0 4096:16 16384:16 16384:64 65536:64 65536:256 262144:64 4096:64 0:0 > $O/sweep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.txt
