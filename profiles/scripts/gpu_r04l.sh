# round 4 final check at HEAD: the whole GPU suite and smoke, the default bench line (what the driver runs), a
# rocprofv3 kernel trace of it, separate FETCH_SIZE / WRITE_SIZE passes of the C3 launch, the C2 / C5 lines, and
# two ranks sharing the one GPU (gloo plumbing rehearsal of --gpus 2 for C3 and C5; not a scaling number)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04l}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -v "^Extension" gpurun_out/${TAG}_pytest_gpu.log | tail -40; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); r=d['roofline']; s=r['single_launch_ring']; print('bench', round(d['value']/1e9,2), 'G frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), 'ws/mall', round(r['working_set_over_mall'],2), 'ring', round(s['frac'],3), 'api', round(d['api_e2e']['value']/1e6,1), 'M', 'cpu', round(d['cpu_baseline']['value']), d['parity'])"
for W in c2 c5; do
  timeout -k 10 300 python bench.py --workload $W --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_$W.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$W.json')); print('$W', d['value'], d['unit'], round(d.get('ms_per_step') or 0, 4))"
done
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-api-e2e --no-ring-roofline > gpurun_out/${TAG}_c3_world2.json 2> gpurun_out/${TAG}_c3_world2.err \
  || { tail -20 gpurun_out/${TAG}_c3_world2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_world2.json')); print('c3 world2 (one GPU)', d['n_gpus'], round(d['value']/1e9,2), 'G', d['parity']['ok'])"
timeout -k 10 400 python bench.py --gpus 2 --workload c5 --steps 10 --warmup 3 > gpurun_out/${TAG}_c5_world2.json 2> gpurun_out/${TAG}_c5_world2.err \
  || { tail -20 gpurun_out/${TAG}_c5_world2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c5_world2.json')); print('c5 world2 (one GPU)', d['n_gpus'], round(d['value']/1e9,3), 'G', d['parity']['ok'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > "$ROOT/gpurun_out/prof_$TAG.json" 2> "$ROOT/gpurun_out/prof_$TAG.err" \
  || { echo "trace pass failed"; tail -20 "$ROOT/gpurun_out/prof_$TAG.err"; exit 1; }
grep -h "pgm_rows_ring\|pgm_rows_jit2" "$ROOT"/gpurun_out/prof_$TAG/*kernel_stats.csv
for W in fetch write; do
  C=$([ $W = fetch ] && echo FETCH_SIZE || echo WRITE_SIZE)
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$ROOT/gpurun_out/pmc_${W}_$TAG" -o p --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-ring-roofline > "$ROOT/gpurun_out/pmc_${W}_$TAG.json" 2> "$ROOT/gpurun_out/pmc_${W}_$TAG.err" \
    || { echo "pmc $C failed"; tail -5 "$ROOT/gpurun_out/pmc_${W}_$TAG.err"; exit 1; }
done
cd "$ROOT"
echo pmc done
