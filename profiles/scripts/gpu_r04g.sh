# round 4 checkpoint: the whole GPU suite and smoke at HEAD, the default bench line (what the driver runs),
# a rocprofv3 kernel trace of it, and separate FETCH_SIZE / WRITE_SIZE passes of the C3 launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04g}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -v "^Extension" gpurun_out/${TAG}_pytest_gpu.log | tail -40; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); r=d['roofline']; s=r['single_launch_ring']; print('bench', round(d['value']/1e9,2), 'G frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), 'ws/mall', round(r['working_set_over_mall'],2), 'ring', round(s['frac'],3), 'api', round(d['api_e2e']['value']/1e6,1), 'M', 'cpu', round(d['cpu_baseline']['value']), d['parity'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > "$ROOT/gpurun_out/prof_$TAG.json" 2> "$ROOT/gpurun_out/prof_$TAG.err" \
  || { echo "trace pass failed"; tail -20 "$ROOT/gpurun_out/prof_$TAG.err"; exit 1; }
grep -h "pgm_rows_ring\|pgm_rows_jit2" "$ROOT"/gpurun_out/prof_$TAG/*kernel_stats.csv
# counters of the C3 launch, one pass each (summarised in the build container: tools/pmc_summary.py TAG pgm_rows_jit2)
for W in fetch write; do
  C=$([ $W = fetch ] && echo FETCH_SIZE || echo WRITE_SIZE)
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$ROOT/gpurun_out/pmc_${W}_$TAG" -o p --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-ring-roofline > "$ROOT/gpurun_out/pmc_${W}_$TAG.json" 2> "$ROOT/gpurun_out/pmc_${W}_$TAG.err" \
    || { echo "pmc $C failed"; tail -5 "$ROOT/gpurun_out/pmc_${W}_$TAG.err"; exit 1; }
done
echo pmc done
for W in c2 c1; do
  for R in 1 2; do
    timeout -k 10 300 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_${W}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_$R.json')); print('$W', round(d['value']*1e3,4), 'ms/query')"
  done
done
timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps.txt 2>&1 && grep "steps," gpurun_out/${TAG}_c2_steps.txt
for MODE in separate same; do
  for OUT in map marginals; do
    PGM_HOST_DELIVERY=$MODE timeout -k 10 300 python bench.py --workload c5 --c5-output $OUT --steps 50 --warmup 5 > gpurun_out/${TAG}_c5_${MODE}_$OUT.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_c5_${MODE}_$OUT.json')); print('c5 $MODE $OUT', round(d['value']/1e9,3), 'G rows/s', 'ms/step', round(d['ms_per_step'],3), 'copy', round(d['copy_ms'],3), d['parity']['ok'])"
  done
done
