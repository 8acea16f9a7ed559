# round 3: C4 schedule depth — fused small clique passes (PGM_MARG_MIN_BLOCKS) and collect messages from
# unaggregated operands (PGM_BP_DIRECT_OPS): parity + A/B at 1,000 / 4,000 rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03ad}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_kernels_gpu.py -k "bp or belief or calibrat or pathfinder or jt or product_n" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 1 2; do
for MB in 512 64; do
for DO in 0 1; do
for ROWS in 1000 4000; do
PGM_MARG_MIN_BLOCKS=$MB PGM_BP_DIRECT_OPS=$DO timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_m${MB}_d${DO}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_m${MB}_d${DO}_$R.json')); print('c4 rows $ROWS min_blocks $MB direct $DO', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
done
done
done
