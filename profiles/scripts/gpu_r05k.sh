# r05k: specialised batches with gather jobs: C1 / C2 / compiled-query parity, then C2 / C1 rates
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05k
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_hazards_gpu.py tests/test_plan_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05k/pytest.log 2>&1 \
  || { echo pytest failed; tail -60 gpurun_out/r05k/pytest.log; exit 1; }
tail -3 gpurun_out/r05k/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05k/c2_$i.json 2> gpurun_out/r05k/c2.err || { tail -20 gpurun_out/r05k/c2.err; exit 1; }
  timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 20 > gpurun_out/r05k/c1_$i.json 2> gpurun_out/r05k/c1.err || { tail -20 gpurun_out/r05k/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05k/c2_$i.json')); e=json.load(open('gpurun_out/r05k/c1_$i.json')); print('c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
done
timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/r05k/c2_steps.txt 2>&1; tail -22 gpurun_out/r05k/c2_steps.txt
