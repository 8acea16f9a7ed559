# r05w: the public API's direct path overlapped with the NaN scan (speculative), parity + api_e2e
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "direct_path or categorical or headline or predict" > gpurun_out/r05w/t0.log 2>&1 || { tail -40 gpurun_out/r05w/t0.log; exit 1; }
tail -3 gpurun_out/r05w/t0.log
timeout -k 10 300 python -u tools/e2e_profile.py > gpurun_out/r05w/e2e.log 2>&1 || { tail -20 gpurun_out/r05w/e2e.log; exit 1; }
tail -12 gpurun_out/r05w/e2e.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-c5 --no-cpu-baseline --no-ring-roofline > gpurun_out/r05w/c3_$i.json 2> gpurun_out/r05w/c3.err || { tail -20 gpurun_out/r05w/c3.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05w/c3_$i.json')); print('api_e2e', round(d['api_e2e']['value']/1e6,2), 'M rows/s', round(d['api_e2e']['seconds']*1e3,3), 'ms')"
done
