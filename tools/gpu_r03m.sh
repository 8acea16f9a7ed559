# round 3: C4 clique layout (shared separator variables slowest) A/B + BP parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03m}
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
for LY in 1 0 1 0; do
for R in 4000 1000; do
PGM_BP_LAYOUT=$LY timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${R}_ly$LY.json 2> gpurun_out/${TAG}_c4_${R}_ly$LY.err || { tail -30 gpurun_out/${TAG}_c4_${R}_ly$LY.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${R}_ly$LY.json')); print('layout $LY rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms', round(d['frac_of_8TBps'],3))"
done
done
timeout -k 10 900 $T -m gpu tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_markov.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -60 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
LEVELS=1 TOP=8 timeout -k 10 300 python tools/program_steps.py c4 4000 > gpurun_out/${TAG}_c4_levels.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c4_levels.txt; exit 1; }
head -2 gpurun_out/${TAG}_c4_levels.txt; grep -A2 "^-- level 2[2-3]" gpurun_out/${TAG}_c4_levels.txt | cut -c1-150
