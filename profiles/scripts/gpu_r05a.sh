# r05a: the new parity tests (C4 bench schedule, wide evidence, threaded BP), then the default bench
# line (with the C5 sub-object) and the C4 line with its parity field.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "c4_bench_schedule or wide_evidence or threads_share_one_belief" > gpurun_out/r05a/pytest_new.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05a/pytest_new.log; exit 1; }
tail -5 gpurun_out/r05a/pytest_new.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err \
  || { echo bench failed; tail -30 gpurun_out/r05a/bench.err; exit 1; }
tail -c 3000 gpurun_out/r05a/bench.json
timeout -k 10 300 python -u bench.py --workload c4 --rows 4000 --steps 10 --warmup 3 > gpurun_out/r05a/c4.json 2> gpurun_out/r05a/c4.err \
  || { echo c4 failed; tail -30 gpurun_out/r05a/c4.err; exit 1; }
cat gpurun_out/r05a/c4.json
