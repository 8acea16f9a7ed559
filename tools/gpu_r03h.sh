# round 3: C3 direct with the parallel in-window release (x3), ring with / without prestart, the driver
# config under a rocprofv3 kernel trace (the window's span from the trace), sampling + stochastic tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03h}
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_inference_gpu.py -k "stochastic or sample_joint" > gpurun_out/${TAG}_pytest_sample.log 2>&1 || { echo sample tests failed; tail -60 gpurun_out/${TAG}_pytest_sample.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_sample.log
timeout -k 10 300 $T tests/test_plan_gpu.py -k "direct or ring" > gpurun_out/${TAG}_pytest_dq.log 2>&1 || { echo dq tests failed; tail -60 gpurun_out/${TAG}_pytest_dq.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_dq.log
for R in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench_direct20_$R.json 2> gpurun_out/${TAG}_bench_direct20_$R.err || { tail -30 gpurun_out/${TAG}_bench_direct20_$R.err; exit 1; }
timeout -k 10 300 python bench.py --launch ring --ring-prestart --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench_ringpre20_$R.json 2> gpurun_out/${TAG}_bench_ringpre20_$R.err || { tail -30 gpurun_out/${TAG}_bench_ringpre20_$R.err; exit 1; }
timeout -k 10 300 python bench.py --launch ring --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench_ring20_$R.json 2> gpurun_out/${TAG}_bench_ring20_$R.err || { tail -30 gpurun_out/${TAG}_bench_ring20_$R.err; exit 1; }
done
timeout -k 10 300 python bench.py --launch ring --ring-prestart --steps 400 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench_ringpre400.json 2> gpurun_out/${TAG}_bench_ringpre400.err || { tail -30 gpurun_out/${TAG}_bench_ringpre400.err; exit 1; }
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d.get("roofline") or {}
    print(f.split("/")[-1], round(d["value"]/1e9,2), "G", round(d["ms_per_step"]*1e3,3), "us", {k: (round(r[k],3) if isinstance(r.get(k), float) else r.get(k)) for k in ("frac","frac_wall","kernel_ms")}, (d.get("parity") or {}).get("ok"))'
python -c "$P" gpurun_out/${TAG}_bench_*.json
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof_direct -o direct -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench_direct20_prof.json 2> gpurun_out/${TAG}_bench_direct20_prof.err || { tail -30 gpurun_out/${TAG}_bench_direct20_prof.err; exit 1; }
TR=$(find gpurun_out/${TAG}_prof_direct -name "*kernel_trace.csv" | head -1)
python tools/trace_span.py "$TR" gpurun_out/${TAG}_bench_direct20_prof.json > gpurun_out/${TAG}_trace_span_direct.json && cat gpurun_out/${TAG}_trace_span_direct.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_ring -o ring -- python3 bench.py --launch ring --ring-prestart --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_bench_ringpre20_prof.json 2> gpurun_out/${TAG}_bench_ringpre20_prof.err || { tail -30 gpurun_out/${TAG}_bench_ringpre20_prof.err; exit 1; }
find gpurun_out/${TAG}_prof_ring -name "*kernel_stats.csv" -exec head -5 {} \;
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail -30 gpurun_out/${TAG}_bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); print(d['value'], d['roofline']['frac'], d['roofline']['frac_wall'], d.get('api_e2e'), d.get('cpu_baseline',{}).get('value'))"
