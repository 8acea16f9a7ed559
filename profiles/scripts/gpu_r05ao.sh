# r05ao: every single query through the steps program (fused plans too): parity suites, C1 / C2, alarm probe
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05ao
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_plan_gpu.py tests/test_compat_gpu.py > gpurun_out/r05ao/t0.log 2>&1 || { tail -40 gpurun_out/r05ao/t0.log; exit 1; }
tail -1 gpurun_out/r05ao/t0.log
timeout -k 10 300 python -u tools/alarm_marg_probe.py 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c1 --steps 300 --warmup 30 > gpurun_out/r05ao/c1_$i.json 2> gpurun_out/r05ao/c1.err || { tail -20 gpurun_out/r05ao/c1.err; exit 1; }
  timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05ao/c2_$i.json 2> gpurun_out/r05ao/c2.err || { tail -20 gpurun_out/r05ao/c2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05ao/c2_$i.json')); e=json.load(open('gpurun_out/r05ao/c1_$i.json')); print('c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
done
