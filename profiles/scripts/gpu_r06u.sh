# r06u: C1 / C2 single queries split into the AQL chains and the Python part, with a cProfile of the latter
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/query_split.py 200 > $O/split.txt 2> $O/split.err || { tail -30 $O/split.err; exit 1; }
tail -1 $O/split.txt
