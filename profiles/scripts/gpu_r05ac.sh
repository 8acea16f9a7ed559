# r05ac: C4 marginal-only passes walk a psi-only kept dim inside the block (PGM_PM_TILE A/B), parity
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05ac
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "psi_tile or product_n or two_marginals or bp_levelled" > gpurun_out/r05ac/t0.log 2>&1 || { tail -40 gpurun_out/r05ac/t0.log; exit 1; }
tail -2 gpurun_out/r05ac/t0.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "pathfinder or bp or belief" > gpurun_out/r05ac/t1.log 2>&1 || { tail -40 gpurun_out/r05ac/t1.log; exit 1; }
tail -2 gpurun_out/r05ac/t1.log
for i in 1 2; do for X in 1 0; do for R in 4000 1000; do
  PGM_PM_TILE=$X timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05ac/c4_${X}_${R}_$i.json 2> gpurun_out/r05ac/c4.err || { tail -20 gpurun_out/r05ac/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05ac/c4_${X}_${R}_$i.json')); print('tile=$X', $R, round(d['value']/1e6,4), 'M/s one', round(d['one_in_flight']['value']/1e6,4), d['parity']['ok'])"
done; done; done
