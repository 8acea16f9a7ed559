# C3 under the 4-queue default: workgroup size (PGM_ROWS_JIT_WG) x row form (one row / two rows per
# thread), then one rocprofv3 kernel trace of the default bench for the per-dispatch comparison
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
P='import json,sys
d=json.load(open(sys.argv[1])); r=d.get("roofline") or {}
print(sys.argv[2], "value=%.3g" % d["value"], "ms/step=%.5f" % d["ms_per_step"], "frac=%.3f" % (r.get("frac") or 0), "kernel_ms=%s" % r.get("kernel_ms"), "dispatch_avg_ms=%s" % r.get("dispatch_avg_ms"), "floor=%s" % r.get("dispatch_floor_ms"))'
for steps in 400 20; do
for wg in 256 128 512 1024; do
for j2 in 400000 50000; do
  T="wg${wg}_j2${j2}_s${steps}"
  PGM_ROWS_JIT_WG=$wg PGM_JIT2_MIN_ROWS=$j2 timeout -k 10 200 python bench.py --steps $steps --warmup 10 --no-cpu-baseline > gpurun_out/sw_$T.json 2> gpurun_out/sw_$T.err || { tail -20 gpurun_out/sw_$T.err; exit 1; }
  python -c "$P" gpurun_out/sw_$T.json $T
done
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_sw" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$ROOT/gpurun_out/prof_sw.json" 2> "$ROOT/gpurun_out/prof_sw.err" || { tail -20 "$ROOT/gpurun_out/prof_sw.err"; exit 1; }
cd "$ROOT" && python -c "$P" gpurun_out/prof_sw.json under_rocprof
cat gpurun_out/prof_sw/trace_kernel_stats.csv | cut -c1-200
