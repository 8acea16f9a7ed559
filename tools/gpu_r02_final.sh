# round-2 evidence (+ single-queue rocprof pass): GPU suite, smoke, C3 (20 and 400 steps), C5 N=1, C1, C2, C4 (1000/4000), N=2 self-launch, rocprof+PMC of C3
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || { tail -30 gpurun_out/${TAG}_bench_c3.err; exit 1; }
cat gpurun_out/${TAG}_bench_c3.json
timeout -k 10 300 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_bench_c3_400.json 2> gpurun_out/${TAG}_bench_c3_400.err || { tail -30 gpurun_out/${TAG}_bench_c3_400.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.err || { tail -30 gpurun_out/${TAG}_bench_c5.err; exit 1; }
timeout -k 10 300 python bench.py --workload c1 --steps 100 --warmup 2 > gpurun_out/${TAG}_bench_c1.json 2> gpurun_out/${TAG}_bench_c1.err || { tail -30 gpurun_out/${TAG}_bench_c1.err; exit 1; }
timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { tail -30 gpurun_out/${TAG}_bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --workload c4 --rows 1000 --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_c4_1000.json 2> gpurun_out/${TAG}_bench_c4_1000.err || { tail -30 gpurun_out/${TAG}_bench_c4_1000.err; exit 1; }
timeout -k 10 300 python bench.py --workload c4 --rows 4000 --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_c4_4000.json 2> gpurun_out/${TAG}_bench_c4_4000.err || { tail -30 gpurun_out/${TAG}_bench_c4_4000.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_n2.json 2> gpurun_out/${TAG}_bench_n2.err || { tail -30 gpurun_out/${TAG}_bench_n2.err; exit 1; }
timeout -k 10 300 python tools/e2e_predict.py 100000 > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -30 gpurun_out/${TAG}_e2e.err; exit 1; }
P='import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); print(f, {k: d.get(k) for k in ("value","unit","ms_per_step")}, (d.get("roofline") or {}).get("frac"))'
python -c "$P" gpurun_out/${TAG}_bench_*.json
bash tools/gpu_profile.sh ${TAG} --steps 200 --warmup 10 || exit 1
# one batch on one queue under rocprofv3 (no overlapping dispatches): rocprof's per-kernel average beside
# the same run's single-queue figures
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_q1_${TAG}" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --steps 200 --warmup 10 --batches 1 --queues 1 > "$ROOT/gpurun_out/prof_q1_${TAG}.json" 2> "$ROOT/gpurun_out/prof_q1_${TAG}.err" || { tail -20 "$ROOT/gpurun_out/prof_q1_${TAG}.err"; exit 1; }
cd "$ROOT"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 10 --batches 1 --queues 1 > gpurun_out/${TAG}_bench_c3_q1.json 2> gpurun_out/${TAG}_bench_c3_q1.err || { tail -20 gpurun_out/${TAG}_bench_c3_q1.err; exit 1; }
echo q1 done
