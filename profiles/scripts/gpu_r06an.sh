# r06an: the public API's direct path split into stages (tools/e2e_direct_stages.py)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06an; mkdir -p $O
export TMPDIR=/tmp
nproc > $O/nproc.txt
timeout -k 10 300 python -u tools/e2e_direct_stages.py 30 > $O/stages.json 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
cat $O/stages.json
