# r06af: C2's program at the new fusion defaults (512 Ki / 512), per level and per launch replayed alone
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06af; mkdir -p $O
export TMPDIR=/tmp FUSED_ONLY=1
timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
cat $O/levels.txt
