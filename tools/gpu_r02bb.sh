# dispatch-floor kernel: its GPU test, C3 at 20 / 400 steps with the floor beside the kernel; C4 per-level and per-step (unmerged) listing at 4000 rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_plan_gpu.py -k "floor or bound or direct" -x -v --timeout 120 --timeout-method thread > gpurun_out/bb_pytest.log 2>&1 || { tail -40 gpurun_out/bb_pytest.log; exit 1; }
tail -2 gpurun_out/bb_pytest.log
for K in 20 400; do
$T 300 python bench.py --steps $K --warmup 5 --no-cpu-baseline > gpurun_out/bb_c3_$K.json 2> gpurun_out/bb_c3_$K.err || { tail -30 gpurun_out/bb_c3_$K.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[1],d['value']/1e9,d['ms_per_step']*1e3,r['kernel_ms']*1e3,r['dispatch_floor_ms']*1e3,r['kernel_over_floor'])" gpurun_out/bb_c3_$K.json
done
LEVELS=1 TOP=0 $T 300 python -u tools/program_steps.py c4 4000 > gpurun_out/bb_c4_levels_4000.txt 2>&1 || { tail -30 gpurun_out/bb_c4_levels_4000.txt; exit 1; }
PGM_PM_MERGE=0 LEVELS=1 TOP=0 $T 300 python -u tools/program_steps.py c4 4000 full > gpurun_out/bb_c4_steps_4000.txt 2>&1 || { tail -30 gpurun_out/bb_c4_steps_4000.txt; exit 1; }
grep -- "-- level\|total\|steps," gpurun_out/bb_c4_levels_4000.txt
