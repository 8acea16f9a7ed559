# direct AQL launch A/B: acquire x release fence scope, C3 400 steps (wall per step + GPU span); parity tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -k "direct" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dq.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_dq.log; exit 1; }
tail -1 gpurun_out/pytest_dq.log
for A in none agent; do for R in none agent system; do
PGM_DQ_ACQ=$A PGM_DQ_REL=$R timeout -k 10 300 python bench.py --steps 400 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${A}_$R.json 2> gpurun_out/ab_${A}_$R.err || { tail -30 gpurun_out/ab_${A}_$R.err; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value']/1e9,'G rows/s',d['ms_per_step']*1e3,'us/step kern',d['roofline']['kernel_ms']*1e3,'us parity',d['parity']['ok'])" gpurun_out/ab_${A}_$R.json
done; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_default_20.json 2> gpurun_out/ab_default_20.err || { tail -30 gpurun_out/ab_default_20.err; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value']/1e9,'G rows/s',d['ms_per_step']*1e3,'us/step kern',d['roofline']['kernel_ms']*1e3,'us parity',d['parity']['ok'])" gpurun_out/ab_default_20.json
