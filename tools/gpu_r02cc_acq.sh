# C3 at 20 steps: each queue's first (system-scope acquire) dispatch before the timed window (default)
# vs inside it (--acquire-in-window), interleaved repeats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1])); r=d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.5f" % d["ms_per_step"], "frac=%.3f" % (r.get("frac") or 0), "kernel_ms=%.5f" % (r.get("kernel_ms") or 0), "parity=%s" % d["parity"]["ok"])'
for rep in 1 2 3 4 5; do
for cfg in default --acquire-in-window; do
  T="${cfg#--}_$rep"
  A=""; [ $cfg != default ] && A=$cfg
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $A > gpurun_out/acq_$T.json 2> gpurun_out/acq_$T.err || { tail -20 gpurun_out/acq_$T.err; exit 1; }
  python -c "$P" gpurun_out/acq_$T.json $T
done
done
