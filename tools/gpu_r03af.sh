# round 3: C4 short-reduction fused passes on few blocks + raw operand folding (PGM_BP_FOLD_RAW): parity + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03af}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_markov.py tests/test_factor_graph.py -k "bp or belief or calibrat or pathfinder or jt or product_n or markov or junction" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 1 2; do
for FR in 4 0; do
for ROWS in 1000 4000; do
PGM_BP_FOLD_RAW=$FR timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_f${FR}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_f${FR}_$R.json')); print('c4 rows $ROWS fold_raw $FR', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
done
done
