# r06ai: C2 / C1 with level batches cut into kernels of at most PGM_PART_JOBS jobs (independent packets of one
# level): is a wide level's time per-kernel (code size, dispatch tree) or aggregate?
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ai; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for PJ in 0 32 16 8; do
  PGM_PART_JOBS=$PJ timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_${PJ}_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  echo "part_jobs $PJ"; cat $O/sweep_${PJ}_$rep.txt
done
done
