# round 3: C4 clique layout for the large cliques only (threshold A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03n}
for CFG in "1 16384" "0 0" "1 30000" "1 8000" "1 16384" "0 0"; do
set -- $CFG; LY=$1; MN=$2
for R in 4000 1000; do
PGM_BP_LAYOUT=$LY PGM_BP_LAYOUT_MIN=$MN timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${R}_ly${LY}_$MN.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${R}_ly${LY}_$MN.json')); print('layout $LY min $MN rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
done
PGM_BP_LAYOUT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_inference_gpu.py -k "pathfinder or bp or belief" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
