# after the C4 row-pair minimum: BP / batched-BP GPU tests, then C4 at 1,000 / 4,000 rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/bx_pytest.log 2>&1 || { tail -40 gpurun_out/bx_pytest.log; exit 1; }
tail -1 gpurun_out/bx_pytest.log
for rows in 1000 4000; do
  timeout -k 10 200 python bench.py --workload c4 --rows $rows --steps 20 --warmup 3 > gpurun_out/r02bx_bench_c4_$rows.json 2> gpurun_out/r02bx_bench_c4_$rows.err || { tail -20 gpurun_out/r02bx_bench_c4_$rows.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r02bx_bench_c4_$rows.json')); print($rows, d['value'], d['ms_per_step'])"
done
