# C3: HIP's own hardware queues (GPU_MAX_HW_QUEUES, default 4) vs the bench's user-mode queues
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1])); r=d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.5f" % d["ms_per_step"], "frac=%.3f" % (r.get("frac") or 0), "kernel_ms=%.5f" % (r.get("kernel_ms") or 0))'
for hq in 4 1 2; do
for q in 4 6; do
for s in 20 20 400; do
  T="hq${hq}_q${q}_s${s}_$RANDOM"
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 200 python bench.py --steps $s --warmup 5 --queues $q --no-cpu-baseline > gpurun_out/hq_$T.json 2> gpurun_out/hq_$T.err || { tail -20 gpurun_out/hq_$T.err; exit 1; }
  python -c "$P" gpurun_out/hq_$T.json $T
done
done
done
