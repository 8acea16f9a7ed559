# r06ac: C2's program at fusion budget 256 Ki / 512 summed entries (split n-ary walks), per level and per launch
# replayed alone; the same with 4x the lanes per n-ary job (PGM_BATCH_LANES_CAP=16384)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ac; mkdir -p $O
export TMPDIR=/tmp FUSED_ONLY=1
timeout -k 10 300 python -u tools/c2_fuse_levels.py 262144 512 > $O/levels_256k.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
cat $O/levels_256k.txt
PGM_BATCH_LANES_CAP=16384 timeout -k 10 300 python -u tools/c2_fuse_levels.py 262144 512 > $O/levels_256k_lanes.txt 2>> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels_256k_lanes.txt
PGM_BATCH_LANES_CAP=16384 timeout -k 10 500 python tools/fuse_sweep.py 65536:64 262144:512 1048576:512 > $O/sweep_lanes.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep_lanes.txt
