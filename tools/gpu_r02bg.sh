# timed region ends on queue completion (timestamps read after it): default C3 x3 at 20 steps, 400 steps, 24-batch variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d["roofline"]; h=r.get("hbm_stream") or {}
    print(f, d["n_gpus"], round(d["value"]/1e9,2), "G/s", round(d["ms_per_step"]*1e3,3), "us/step kern", round(r["kernel_ms"]*1e3,3), "frac", round(r["frac"],3), "stream", h.get("kernel_ms") and round(h["kernel_ms"]*1e3,3), h.get("frac") and round(h["frac"],3), d.get("parity",{}).get("ok"))'
for i in 1 2 3; do
$T 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bg_c3_20_$i.json 2> gpurun_out/bg_c3_20_$i.err || { tail -30 gpurun_out/bg_c3_20_$i.err; exit 1; }
done
$T 300 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/bg_c3_400.json 2> gpurun_out/bg_c3_400.err || { tail -30 gpurun_out/bg_c3_400.err; exit 1; }
$T 300 python bench.py --steps 20 --warmup 5 --batches 1 --queues 1 --no-cpu-baseline > gpurun_out/bg_c3_b1q1_20.json 2> gpurun_out/bg_c3_b1q1_20.err || { tail -30 gpurun_out/bg_c3_b1q1_20.err; exit 1; }
$T 300 python bench.py --steps 20 --warmup 5 --batches 24 --queues 4 --no-cpu-baseline > gpurun_out/bg_c3_b24q4_20.json 2> gpurun_out/bg_c3_b24q4_20.err || { tail -30 gpurun_out/bg_c3_b24q4_20.err; exit 1; }
$T 300 python bench.py --steps 400 --warmup 5 --batches 24 --queues 4 --no-cpu-baseline > gpurun_out/bg_c3_b24q4_400.json 2> gpurun_out/bg_c3_b24q4_400.err || { tail -30 gpurun_out/bg_c3_b24q4_400.err; exit 1; }
$T 300 python bench.py --steps 20 --warmup 5 --launch hip --no-cpu-baseline > gpurun_out/bg_c3_hip.json 2> gpurun_out/bg_c3_hip.err || { tail -30 gpurun_out/bg_c3_hip.err; exit 1; }
python3 -c "$P" gpurun_out/bg_c3_*.json
