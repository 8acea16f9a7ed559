# C3 default = 24 resident batches (343 MB > MALL) on 4 queues: bench 20 steps (with CPU baseline) x2, 400 steps, b4 comparison, --gpus 2; rocprof + PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
TAG=r02bh
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d["roofline"]; h=r.get("hbm_stream") or {}
    print(f, d["n_gpus"], round(d["value"]/1e9,2), "G/s", round(d["ms_per_step"]*1e3,3), "us/step kern", round(r["kernel_ms"]*1e3,3), "frac", round(r["frac"],3), "ws>mall", r.get("working_set_exceeds_mall"), "stream", h.get("kernel_ms") and round(h["kernel_ms"]*1e3,3), h.get("frac") and round(h["frac"],3), d.get("parity",{}).get("ok"))'
$T 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || { tail -30 gpurun_out/${TAG}_bench_c3.err; exit 1; }
$T 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_c3_b.json 2> gpurun_out/${TAG}_bench_c3_b.err || { tail -30 gpurun_out/${TAG}_bench_c3_b.err; exit 1; }
$T 300 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_bench_c3_400.json 2> gpurun_out/${TAG}_bench_c3_400.err || { tail -30 gpurun_out/${TAG}_bench_c3_400.err; exit 1; }
$T 300 python bench.py --steps 20 --warmup 5 --batches 4 --no-cpu-baseline > gpurun_out/${TAG}_bench_c3_b4.json 2> gpurun_out/${TAG}_bench_c3_b4.err || { tail -30 gpurun_out/${TAG}_bench_c3_b4.err; exit 1; }
$T 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_n2.json 2> gpurun_out/${TAG}_bench_n2.err || { tail -30 gpurun_out/${TAG}_bench_n2.err; exit 1; }
python3 -c "$P" gpurun_out/${TAG}_bench_*.json
bash tools/gpu_profile.sh ${TAG} --steps 200 --warmup 10 || exit 1
