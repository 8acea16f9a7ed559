# round 3: C4 write-through product stores A/B (graph replay includes the kernel boundaries)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03k}
for WT in 0 1 0 1; do
for R in 4000 1000; do
PGM_PM_WT=$WT timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${R}_wt$WT.json 2> gpurun_out/${TAG}_c4_${R}_wt$WT.err || { tail -30 gpurun_out/${TAG}_c4_${R}_wt$WT.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${R}_wt$WT.json')); print('wt $WT rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms', round(d['frac_of_8TBps'],3))"
done
done
PGM_PM_WT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_inference_gpu.py -k "pathfinder or bp" > gpurun_out/${TAG}_pytest_bp_wt.log 2>&1 || { echo bp tests failed with WT; tail -40 gpurun_out/${TAG}_pytest_bp_wt.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_bp_wt.log
PGM_PM_WT=1 LEVELS=1 TOP=8 timeout -k 10 300 python tools/program_steps.py c4 4000 > gpurun_out/${TAG}_c4_levels_wt.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c4_levels_wt.txt; exit 1; }
head -2 gpurun_out/${TAG}_c4_levels_wt.txt
