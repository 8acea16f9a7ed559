# r05ai: C4 two sigma' from one computed source in one pass (PGM_BP_PAIR A/B), BP parity
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05ai
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_hazards_gpu.py -k "pathfinder or bp or belief or calibrat or hazard or markov" > gpurun_out/r05ai/t0.log 2>&1 || { tail -40 gpurun_out/r05ai/t0.log; exit 1; }
tail -1 gpurun_out/r05ai/t0.log
for i in 1 2; do for X in 1 0; do for R in 4000 1000; do
  PGM_BP_PAIR=$X timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05ai/c4_${X}_${R}_$i.json 2> gpurun_out/r05ai/c4.err || { tail -20 gpurun_out/r05ai/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05ai/c4_${X}_${R}_$i.json')); print('pair=$X', $R, round(d['value']/1e6,4), 'M/s one', round(d['one_in_flight']['value']/1e6,4), d['parity']['ok'], round(d['executed_step_bytes_per_calibration']/1e6,3), 'MB')"
done; done; done
