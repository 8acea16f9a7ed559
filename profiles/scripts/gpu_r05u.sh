# r05u: C3 default line with completion signals only where read (PGM_DQ_SPARSE=1) vs every dispatch
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05u
export TMPDIR=/tmp
PGM_DQ_SPARSE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_plan_gpu.py > gpurun_out/r05u/t0.log 2>&1 || { tail -40 gpurun_out/r05u/t0.log; exit 1; }
tail -2 gpurun_out/r05u/t0.log
for i in 1 2 3; do for X in 0 1; do
  PGM_DQ_SPARSE=$X timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-c5 --no-cpu-baseline --no-api-e2e > gpurun_out/r05u/c3_${X}_$i.json 2> gpurun_out/r05u/c3.err || { tail -20 gpurun_out/r05u/c3.err; exit 1; }
  PGM_DQ_SPARSE=$X timeout -k 10 300 python -u bench.py --steps 400 --warmup 20 --no-c5 --no-cpu-baseline --no-api-e2e --no-ring-roofline > gpurun_out/r05u/c3l_${X}_$i.json 2> gpurun_out/r05u/c3.err || { tail -20 gpurun_out/r05u/c3.err; exit 1; }
  python -c "
import json
for f in ('c3','c3l'):
    d=json.load(open('gpurun_out/r05u/%s_${X}_$i.json'%f)); r=d.get('roofline',{})
    print('sparse=$X', f, round(d['value']/1e9,2), 'G rows/s', 'ms_per_step', round(d['ms_per_step']*1e3,3), 'us', 'frac', r.get('frac'), d.get('parity',{}).get('ok') if isinstance(d.get('parity'),dict) else d.get('parity'))
"
done; done
