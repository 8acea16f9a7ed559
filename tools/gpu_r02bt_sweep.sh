# C3 (two rows per thread): workgroup sizes around 512 (rows per block 768 ... 1,536) and queue counts
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1])); r=d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.5f" % d["ms_per_step"], "frac=%.3f" % (r.get("frac") or 0), "kernel_ms=%.5f" % (r.get("kernel_ms") or 0), "single=%s" % r.get("single_queue_kernel_ms"), "floor=%s" % r.get("dispatch_floor_ms"), "grid=%s" % r.get("grid"))'
run() {  # tag, env..., -- bench args
  T=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline $BARGS > gpurun_out/bt_$T.json 2> gpurun_out/bt_$T.err || { tail -20 gpurun_out/bt_$T.err; exit 1; }
  python -c "$P" gpurun_out/bt_$T.json $T
}
for wg in 384 512 640 768; do
  for r in a b c; do BARGS="--steps 20 --warmup 5" run wg${wg}_s20_$r PGM_ROWS_JIT_WG=$wg || exit 1; done
  BARGS="--steps 400 --warmup 10" run wg${wg}_s400 PGM_ROWS_JIT_WG=$wg || exit 1
done
for q in 2 3 6; do
  for r in a b; do BARGS="--steps 20 --warmup 5 --queues $q" run q${q}_s20_$r PGM_ROWS_JIT_WG=512 || exit 1; done
  BARGS="--steps 400 --warmup 10 --queues $q" run q${q}_s400 PGM_ROWS_JIT_WG=512 || exit 1
done
