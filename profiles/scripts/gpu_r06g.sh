# r06g: where the fused C2 program's time goes (per level jobs and per step times), fused vs not
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/c2_fuse_levels.py > $O/levels.txt 2> $O/levels.err || { tail -20 $O/levels.err; exit 1; }
cat $O/levels.txt
