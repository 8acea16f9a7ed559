# r05h: plan-specialised contraction batches (C1 / C2 path levels): parity, then C2 / C1 A/B
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05h
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_hazards_gpu.py -m gpu -k "c2 or chain or bn6 or alarm or hazard or compiled" -x -v --timeout 300 --timeout-method thread > gpurun_out/r05h/pytest.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05h/pytest.log; exit 1; }
tail -3 gpurun_out/r05h/pytest.log
for i in 1 2; do for X in 0 1; do
  PGM_BATCH_RTC=$X timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05h/c2_${X}_$i.json 2> gpurun_out/r05h/c2.err || { tail -20 gpurun_out/r05h/c2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05h/c2_${X}_$i.json')); print('c2 rtc=$X', round(d['value']*1e3,4), 'ms/query', d['parity']['ok'])"
  PGM_BATCH_RTC=$X timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 20 > gpurun_out/r05h/c1_${X}_$i.json 2> gpurun_out/r05h/c1.err || { tail -20 gpurun_out/r05h/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05h/c1_${X}_$i.json')); print('c1 rtc=$X', round(d['value']*1e3,4), 'ms/query')"
done; done
timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/r05h/c2_steps.txt 2>&1; tail -30 gpurun_out/r05h/c2_steps.txt
