# direct AQL launch: parity tests, then C3 at 20 / 400 steps with both launchers, C5 N=1, rocprof of the direct C3 run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -k "direct or bound" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_dq.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_dq.log; exit 1; }
tail -2 gpurun_out/pytest_dq.log
for L in direct hip; do for K in 20 400; do
timeout -k 10 300 python bench.py --steps $K --warmup 5 --launch $L --no-cpu-baseline > gpurun_out/bench_c3_${L}_$K.json 2> gpurun_out/bench_c3_${L}_$K.err || { tail -30 gpurun_out/bench_c3_${L}_$K.err; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value']/1e9,'G rows/s',d['ms_per_step']*1e3,'us/step kern',d['roofline']['kernel_ms']*1e3,'us')" gpurun_out/bench_c3_${L}_$K.json
done; done
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > gpurun_out/bench_c5_direct.json 2> gpurun_out/bench_c5_direct.err || { tail -30 gpurun_out/bench_c5_direct.err; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value']/1e9,'G rows/s',d['ms_per_step']*1e3,'us/step kern',d['roofline']['kernel_ms']*1e3,'us')" gpurun_out/bench_c5_direct.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_dq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_c3_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_c3_prof.err || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_c3_prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_dq -name "*stats*" | head; f=$(find gpurun_out/prof_dq -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -5 "$f"
true
