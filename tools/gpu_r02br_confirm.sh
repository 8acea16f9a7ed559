# C3 / C5 confirmation of the workgroup x row-form sweep (r02bq): repeated runs per configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1])); r=d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.5f" % d["ms_per_step"], "frac=%.3f" % (r.get("frac") or 0), "kernel_ms=%.5f" % (r.get("kernel_ms") or 0), "dispatch_avg_ms=%s" % r.get("dispatch_avg_ms"))'
for cfg in 256:400000 512:50000 256:50000 1024:400000 512:400000; do
  wg=${cfg%%:*}; j2=${cfg##*:}
  for run in a b c; do
    T="wg${wg}_j2${j2}_c3s20_$run"
    PGM_ROWS_JIT_WG=$wg PGM_JIT2_MIN_ROWS=$j2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cf_$T.json 2> gpurun_out/cf_$T.err || { tail -20 gpurun_out/cf_$T.err; exit 1; }
    python -c "$P" gpurun_out/cf_$T.json $T
  done
  T="wg${wg}_j2${j2}_c3s400"
  PGM_ROWS_JIT_WG=$wg PGM_JIT2_MIN_ROWS=$j2 timeout -k 10 200 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/cf_$T.json 2> gpurun_out/cf_$T.err || { tail -20 gpurun_out/cf_$T.err; exit 1; }
  python -c "$P" gpurun_out/cf_$T.json $T
  T="wg${wg}_j2${j2}_c5s20"
  PGM_ROWS_JIT_WG=$wg PGM_JIT2_MIN_ROWS=$j2 timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cf_$T.json 2> gpurun_out/cf_$T.err || { tail -20 gpurun_out/cf_$T.err; exit 1; }
  python -c "$P" gpurun_out/cf_$T.json $T
  T="wg${wg}_j2${j2}_c3q1"
  PGM_ROWS_JIT_WG=$wg PGM_JIT2_MIN_ROWS=$j2 timeout -k 10 200 python bench.py --steps 400 --warmup 10 --batches 1 --queues 1 --no-cpu-baseline > gpurun_out/cf_$T.json 2> gpurun_out/cf_$T.err || { tail -20 gpurun_out/cf_$T.err; exit 1; }
  python -c "$P" gpurun_out/cf_$T.json $T
done
