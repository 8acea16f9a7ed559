# r06ar: kept-dim reorder (PGM_NARY_KORDER): C2 / C1 timing with and without, then the fused-vs-unfused test with it
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ar; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for KO in 1 0; do
  PGM_NARY_KORDER=$KO timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_${KO}_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  echo "korder $KO"; cat $O/sweep_${KO}_$rep.txt
done
done
PGM_NARY_KORDER=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 300 --timeout-method thread -k "fused_query" > $O/pytest.log 2>&1; tail -3 $O/pytest.log
