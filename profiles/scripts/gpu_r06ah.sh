# r06ah: C2's slow launches (> 4.5 us alone) at the fusion defaults: each of their jobs specialised and replayed alone
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ah; mkdir -p $O
export TMPDIR=/tmp FUSED_ONLY=1 JOB_TIMES=1 DUMP_SRC=gpurun_out/r06ah/src
timeout -k 10 400 python -u tools/c2_fuse_levels.py > $O/levels_jobs.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels_jobs.txt
