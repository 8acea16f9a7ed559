# round 3: C4 balanced product trees (PGM_PRODN_TREE) A/B + BP parity + level profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03q}
for TR in 1 0 1 0; do
for R in 4000 1000; do
PGM_PRODN_TREE=$TR timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${R}_tree$TR.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${R}_tree$TR.json')); print('tree $TR rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
done
for GS in 2 4 1 2; do
for R in 4000 1000; do
PGM_GRAPH_STREAMS=$GS timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${R}_gs$GS.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${R}_gs$GS.json')); print('streams $GS rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
done
PGM_GRAPH_STREAMS=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_inference_gpu.py -k "pathfinder or bp or belief or alarm_bp" > gpurun_out/${TAG}_pytest_dag.log 2>&1 || { echo dag tests failed; tail -40 gpurun_out/${TAG}_pytest_dag.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_dag.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_markov.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
LEVELS=1 TOP=5 timeout -k 10 300 python tools/program_steps.py c4 1000 > gpurun_out/${TAG}_c4_levels_1000.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c4_levels_1000.txt; exit 1; }
head -3 gpurun_out/${TAG}_c4_levels_1000.txt | cut -c1-300
