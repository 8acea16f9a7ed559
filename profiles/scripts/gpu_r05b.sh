# r05b: C2 on the reference's 20 rows (test + bench line with parity)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "munin_c2" > gpurun_out/r05b/pytest_c2.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05b/pytest_c2.log; exit 1; }
tail -5 gpurun_out/r05b/pytest_c2.log
timeout -k 10 300 python -u bench.py --workload c2 --steps 200 --warmup 20 > gpurun_out/r05b/c2.json 2> gpurun_out/r05b/c2.err \
  || { echo c2 failed; tail -30 gpurun_out/r05b/c2.err; exit 1; }
cat gpurun_out/r05b/c2.json
