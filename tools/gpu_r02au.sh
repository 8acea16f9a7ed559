# C3 row kernel: LDS-staged CPT values vs direct global gathers (400 steps, two passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
run() { local lab=$1; shift
  env "$@" $T 300 python -u bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/c3_$lab.json 2> gpurun_out/c3_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c3_$lab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c3_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,3), round(d['roofline']['kernel_ms']*1e3,3), d['parity']['ok'])"
}
for p in 1 2; do
run lds_$p
run nolds_$p PGM_ROWS_JIT_LDS=0
true
done
