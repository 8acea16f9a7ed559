# direct queue: interrupt-free vs event completion signals (write-through stores, no per-dispatch fences)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
P='import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d["value"]/1e9,2),"G rows/s",round(d["ms_per_step"]*1e3,3),"us/step kern",round(d["roofline"]["kernel_ms"]*1e3,3),"us parity",d["parity"]["ok"])'
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -k "direct" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dq.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_dq.log; exit 1; }
tail -1 gpurun_out/pytest_dq.log
for SG in gpu event; do for K in 400 20; do
PGM_DQ_SIGNAL=$SG PGM_ROWS_JIT_STORE=wt PGM_DQ_ACQ=none PGM_DQ_REL=none timeout -k 10 300 python bench.py --steps $K --warmup 5 --no-cpu-baseline > gpurun_out/sig_${SG}_$K.json 2> gpurun_out/sig_${SG}_$K.err || { tail -30 gpurun_out/sig_${SG}_$K.err; exit 1; }
python -c "$P" gpurun_out/sig_${SG}_$K.json
done; done
for K in 400 20; do
PGM_ROWS_JIT_STORE=wt timeout -k 10 300 python bench.py --steps $K --warmup 5 --no-cpu-baseline --launch hip > gpurun_out/sig_hip_$K.json 2> gpurun_out/sig_hip_$K.err || { tail -30 gpurun_out/sig_hip_$K.err; exit 1; }
python -c "$P" gpurun_out/sig_hip_$K.json
done
