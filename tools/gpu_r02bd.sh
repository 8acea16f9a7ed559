# independent row batches on several user-mode queues (CP pipes in parallel): tests, then C3 sweeps at 20 / 400 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_plan_gpu.py -k "queues or group or direct" -x -v --timeout 120 --timeout-method thread > gpurun_out/bd_pytest.log 2>&1 || { tail -40 gpurun_out/bd_pytest.log; exit 1; }
tail -2 gpurun_out/bd_pytest.log
for cfg in "1 1" "2 2" "4 2" "4 4" "8 4" "8 8"; do set -- $cfg
for K in 20 400; do
$T 300 python bench.py --steps $K --warmup 5 --batches $1 --queues $2 --no-cpu-baseline > gpurun_out/bd_c3_b$1_q$2_$K.json 2> gpurun_out/bd_c3_b$1_q$2_$K.err || { tail -30 gpurun_out/bd_c3_b$1_q$2_$K.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[1],round(d['value']/1e9,2),'G/s step',round(d['ms_per_step']*1e3,3),'us kern',round(r['kernel_ms']*1e3,3),'floor',round(r['dispatch_floor_ms']*1e3,3),d['parity']['ok'])" gpurun_out/bd_c3_b$1_q$2_$K.json
done; done
