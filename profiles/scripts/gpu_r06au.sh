# r06au: fusion settings around the new default (512 Ki / 512, critical path only): non-critical absorption,
# 384 Ki, 768 Ki, 768 summed entries (two passes)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06au; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 500 python tools/fuse_sweep.py 524288:512 524288:512:0 393216:512 786432:512 524288:768 > $O/sweep_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep_$rep.txt
done
