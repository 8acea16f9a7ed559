# r06v: C1's programs: launches per chain, steps replayed alone
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c1_programs.py > $O/c1_programs.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
cat $O/c1_programs.txt
