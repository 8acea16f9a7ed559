# C3 at the driver's 20 steps: HIP hardware queues 1 vs 4 (default), interleaved repeats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1])); r=d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.5f" % d["ms_per_step"], "frac=%.3f" % (r.get("frac") or 0), "kernel_ms=%.5f" % (r.get("kernel_ms") or 0))'
for rep in 1 2 3 4 5; do
for hq in 1 4; do
  T="hq${hq}_s20_$rep"
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hz_$T.json 2> gpurun_out/hz_$T.err || { tail -20 gpurun_out/hz_$T.err; exit 1; }
  python -c "$P" gpurun_out/hz_$T.json $T
done
done
for hq in 1 4; do
  T="hq${hq}_c5"
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hz_$T.json 2> gpurun_out/hz_$T.err || { tail -20 gpurun_out/hz_$T.err; exit 1; }
  python -c "$P" gpurun_out/hz_$T.json $T
done
