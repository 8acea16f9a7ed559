# round 5 checkpoint at HEAD: the whole GPU suite and smoke, the default bench line (what the driver runs;
# now with the C5 sub-object), a rocprofv3 kernel trace of it, the C1 / C2 / C4 / C5 lines, C4 per-step PMC
# fetch / write, and two ranks sharing the one GPU (gloo plumbing rehearsal of --gpus 2; not a scaling number)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"
TAG=${1:-r05ck}
mkdir -p gpurun_out/$TAG
O=gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; s=r['single_launch_ring']; c=d['c5']
print('bench', round(d['value']/1e9,2), 'G frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), 'ws/mall', round(r['working_set_over_mall'],2), 'ring', round(s['frac'],3), 'api', round(d['api_e2e']['value']/1e6,1), 'M', 'cpu', round(d['cpu_baseline']['value']), d['parity']['ok'])
print('c5 host', round(c['host']['value']/1e9,3), 'G', 'kernel frac', round(c['host']['roofline']['frac'],3), 'map', round(c['host_map']['value']/1e9,2), 'G', 'rccl', round(c['rccl']['value']/1e9,2), 'G', c['host']['parity']['ok'], c['host_map']['parity']['ok'], c['rccl']['parity']['ok'], 'dma', round(c['host_dma_probe']['one_stream_GBps'],1), round(c['host_dma_probe']['two_streams_full_GBps'],1))"
for W in c1 c2; do
  timeout -k 10 300 python bench.py --workload $W --steps 300 --warmup 30 --no-cpu-baseline > $O/$W.json 2> $O/$W.err || { tail -20 $O/$W.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$W.json')); print('$W', round(d['value']*1e3,4), 'ms/query')"
done
for R in 4000 1000; do
  timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > $O/c4_$R.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_$R.json')); o=d.get('one_in_flight') or {}; print('c4', $R, round(d['value']/1e6,4), 'M/s (inflight', d.get('inflight'), '; one at a time', round((o.get('value') or 0)/1e6,4), ')', d['parity']['ok'], round(d['executed_step_bytes_per_calibration']/1e6,3), 'MB/cal')"
done
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', round(d['value']/1e9,3), 'G rows/s; kernel frac', round(d['roofline']['frac'],3))"
timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-api-e2e --no-ring-roofline > $O/c3_world2.json 2> $O/c3_world2.err \
  || { tail -20 $O/c3_world2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3_world2.json')); c=d['c5']; print('world2 (one GPU)', d['n_gpus'], round(d['value']/1e9,2), 'G', d['parity']['ok'], 'c5 host', round(c['host']['value']/1e9,3), 'G', c['host']['parity']['ok'], 'rccl', round(c['rccl']['value']/1e9,3), c['rccl']['parity']['ok'], c['rows_per_gpu_per_step'])"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/prof" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-c5 > "$ROOT/$O/prof.json" 2> "$ROOT/$O/prof.err" \
  || { echo "trace pass failed"; tail -20 "$ROOT/$O/prof.err"; exit 1; }
grep -h "pgm_rows_ring\|pgm_rows_jit2" "$ROOT"/$O/prof/*kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d "$ROOT/$O/c4pmc_$C" -o p --output-format csv -- \
    python3 "$ROOT/tools/c4_step_pmc.py" run "$ROOT/$O/c4pmc_meta.json" > "$ROOT/$O/c4pmc_$C.log" 2>&1 \
    || { echo "pmc $C failed"; tail -5 "$ROOT/$O/c4pmc_$C.log"; exit 1; }
done
cd "$ROOT"
python3 tools/c4_step_pmc.py summarize $O/c4pmc_meta.json $O/c4pmc_FETCH_SIZE $O/c4pmc_WRITE_SIZE > $O/c4pmc_summary.json
python3 -c "import json; d=json.load(open('$O/c4pmc_summary.json')); print('c4 pmc fetch GB', round(d['fetch_bytes_x2']/1e9,2), 'write GB', round(d['write_bytes']/1e9,2), 'vs floor', round(d['ratio_to_floor'],3))"
