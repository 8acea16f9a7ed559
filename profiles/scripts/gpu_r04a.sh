# round 4: the C3 line over a resident set >= 4x the Infinity Cache (96 batches, 1.37 GB) vs 24 / 48,
# and a rocprofv3 kernel trace of the 96-batch command (ring + jit2 dispatch durations)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04a}
line() {  # file label
  python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; s=r.get('single_launch_ring') or {}; print('$2', round(d['value']/1e9,2), 'G', 'frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), 'ws/mall', round(r['working_set_over_mall'],2), 'ring', round(s.get('frac',0),3), round(s.get('kernel_ms',0),4), 'ring ws/mall', round(s.get('working_set_over_mall',0),2))"
}


timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench96_full.json 2> gpurun_out/${TAG}_bench96_full.err || { tail -30 gpurun_out/${TAG}_bench96_full.err; exit 1; }
line gpurun_out/${TAG}_bench96_full.json b96_full
for B in 24 48 96; do
  for R in 1; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batches $B --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench${B}_$R.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
    line gpurun_out/${TAG}_bench${B}_$R.json b${B}_$R
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > "$ROOT/gpurun_out/prof_$TAG.json" 2> "$ROOT/gpurun_out/prof_$TAG.err" \
  || { echo "trace pass failed"; tail -20 "$ROOT/gpurun_out/prof_$TAG.err"; exit 1; }
cd "$ROOT"
line gpurun_out/prof_$TAG.json profiled
grep -h "pgm_rows_ring\|pgm_rows_jit2" gpurun_out/prof_$TAG/*kernel_stats.csv
