# round 3: single-launch ring roofline in the C3 line + a rocprofv3 kernel trace of the same command
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r03z}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_plan_gpu.py -k "shard or ring" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench20.json 2> gpurun_out/${TAG}_bench20.err || { tail -30 gpurun_out/${TAG}_bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench20.json')); r=d['roofline']; print('c3 20', round(d['value']/1e9,2), round(r['frac'],3), round(r['frac_wall'],3), json.dumps(r['single_launch_ring']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > "$ROOT/gpurun_out/prof_$TAG.json" 2> "$ROOT/gpurun_out/prof_$TAG.err" \
  || { echo "trace pass failed"; tail -20 "$ROOT/gpurun_out/prof_$TAG.err"; exit 1; }
cd "$ROOT"
python -c "import json; d=json.load(open('gpurun_out/prof_${TAG}.json')); print('profiled ring', json.dumps(d['roofline']['single_launch_ring']))"
grep -h "pgm_rows_ring\|pgm_rows_jit2" gpurun_out/prof_$TAG/*kernel_stats.csv
