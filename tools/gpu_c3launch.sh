set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for G in 0 1; do
  if [ $G = 1 ]; then export PGM_BOUND_GRAPH=1; fi
  timeout -k 10 120 python tools/rows_sweep.py --rows 100000 --reps 400 --variants lds_values > gpurun_out/rows_g$G.txt 2>&1; echo "GRAPH=$G $(grep rows gpurun_out/rows_g$G.txt)"
  timeout -k 10 300 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/bench_g$G.json 2> gpurun_out/bench_g$G.err || { tail gpurun_out/bench_g$G.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_g$G.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'])"
done
