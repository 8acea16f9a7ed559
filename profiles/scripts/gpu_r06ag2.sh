# r06ag2: lanes per n-ary job (PGM_NARY_LANES: 4 Ki, 8 Ki, 16 Ki default) at the 512 Ki / 512 fusion defaults
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ag2; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for NL in 4096 8192 16384; do
  PGM_NARY_LANES=$NL timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_${NL}_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  echo "lanes $NL"; cat $O/sweep_${NL}_$rep.txt
done
done
PGM_NARY_LANES=8192 FUSED_ONLY=1 timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels_8k.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels_8k.txt
