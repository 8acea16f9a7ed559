# r06p: C2's fused program at the defaults, per level and per launch replayed alone
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels.txt 2> $O/levels.err || { tail -30 $O/levels.err; exit 1; }
cat $O/levels.txt
