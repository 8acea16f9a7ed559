# C3 (4 queues, two-row kernel): write-through output stores (default) vs plain stores + agent-scope release
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1])); r=d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.5f" % d["ms_per_step"], "frac=%.3f" % (r.get("frac") or 0), "kernel_ms=%.5f" % (r.get("kernel_ms") or 0), "single=%s" % r.get("single_queue_kernel_ms"), "parity=%s" % d["parity"]["ok"])'
for rep in 1 2 3; do
for st in wt plain; do
  T="${st}_s20_$rep"
  PGM_ROWS_JIT_STORE=$st timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/st_$T.json 2> gpurun_out/st_$T.err || { tail -20 gpurun_out/st_$T.err; exit 1; }
  python -c "$P" gpurun_out/st_$T.json $T
done
done
for st in wt plain; do
  T="${st}_s400"
  PGM_ROWS_JIT_STORE=$st timeout -k 10 200 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/st_$T.json 2> gpurun_out/st_$T.err || { tail -20 gpurun_out/st_$T.err; exit 1; }
  python -c "$P" gpurun_out/st_$T.json $T
done
