# C4: nontemporal marginal stores in marginal-only passes (PGM_PM_MNT 1 vs 0), XI auto vs 1; BP parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_inference_gpu.py tests/test_kernels_gpu.py -k "bp or belief or calibrat or product_n or pathfinder" -x -q --timeout 240 --timeout-method thread > gpurun_out/bk_pytest.log 2>&1 || { tail -40 gpurun_out/bk_pytest.log; exit 1; }
tail -1 gpurun_out/bk_pytest.log
for cfg in "1 0" "0 0" "1 1" "0 1"; do set -- $cfg; for R in 4000 1000; do
PGM_PM_MNT=$1 PGM_PM_XI=$2 $T 300 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/bk_c4_${R}_m$1_x$2.json 2> gpurun_out/bk_c4_${R}_m$1_x$2.err || { tail -30 gpurun_out/bk_c4_${R}_m$1_x$2.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']),'cal/s',round(d['ms_per_step'],3),'ms',round(d['frac_of_8TBps'],3))" gpurun_out/bk_c4_${R}_m$1_x$2.json
done; done
LEVELS=1 TOP=0 $T 300 python -u tools/program_steps.py c4 4000 > gpurun_out/bk_c4_levels_4000.txt 2>&1 || { tail -30 gpurun_out/bk_c4_levels_4000.txt; exit 1; }
grep -- "-- level\|total\|steps," gpurun_out/bk_c4_levels_4000.txt | head -8
