# r06ag: lanes per n-ary job (PGM_NARY_LANES: 16 Ki default, 32 Ki, 64 Ki) at the 512 Ki / 512 fusion defaults
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ag; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for NL in 16384 32768 65536; do
  PGM_NARY_LANES=$NL timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_${NL}_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  echo "lanes $NL"; cat $O/sweep_${NL}_$rep.txt
done
done
PGM_NARY_LANES=65536 FUSED_ONLY=1 timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels_64k.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels_64k.txt
