# round 3: C4 investigation — kept-dim tile order A/B (PGM_PM_KREV), unmerged step profile of the root
# levels, PMC HBM traffic of a 4,000-row calibration
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03i}
for KR in 0 1 0 1; do
for R in 4000 1000; do
PGM_PM_KREV=$KR timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${R}_krev$KR.json 2> gpurun_out/${TAG}_c4_${R}_krev$KR.err || { tail -30 gpurun_out/${TAG}_c4_${R}_krev$KR.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${R}_krev$KR.json')); print('krev $KR rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms', round(d['frac_of_8TBps'],3))"
done
done
PGM_PM_MERGE=0 LEVELS=1 TOP=12 timeout -k 10 300 python tools/program_steps.py c4 4000 > gpurun_out/${TAG}_c4_levels_nomerge.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c4_levels_nomerge.txt; exit 1; }
PGM_PM_KREV=1 PGM_PM_MERGE=0 LEVELS=1 TOP=12 timeout -k 10 300 python tools/program_steps.py c4 4000 > gpurun_out/${TAG}_c4_levels_nomerge_krev.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c4_levels_nomerge_krev.txt; exit 1; }
grep -A4 "^-- level 2[2-5]" gpurun_out/${TAG}_c4_levels_nomerge.txt | cut -c1-200
grep -A4 "^-- level 2[2-5]" gpurun_out/${TAG}_c4_levels_nomerge_krev.txt | cut -c1-200
