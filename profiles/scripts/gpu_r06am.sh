# r06am: n-ary jobs' kept dims decoded with the cheapest-to-read dim fastest (PGM_NARY_KORDER=1) vs the output's
# order (0): n-ary tests under both, then C2 / C1 (two passes) and per-launch times
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06am; mkdir -p $O
export TMPDIR=/tmp
PGM_NARY_KORDER=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "contract_n or fused_query or munin_c2 or alarm" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for KO in 1 0; do
  PGM_NARY_KORDER=$KO timeout -k 10 300 python tools/fuse_sweep.py 524288:512 > $O/sweep_${KO}_$rep.txt 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  echo "korder $KO"; cat $O/sweep_${KO}_$rep.txt
done
done
PGM_NARY_KORDER=1 FUSED_ONLY=1 timeout -k 10 300 python -u tools/c2_fuse_levels.py > $O/levels.txt 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
grep -v "^  level" $O/levels.txt
