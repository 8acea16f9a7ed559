# round 3: single-workgroup chains of tiny levels (C1 / C2 tails): parity + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03aa}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "single_workgroup or levelled" > gpurun_out/${TAG}_pytest_k.log 2>&1 || { echo kernel tests failed; tail -40 gpurun_out/${TAG}_pytest_k.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_k.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_markov.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 1 2; do
for W in 4 0; do
PGM_WG_CHAIN_BLOCKS=$W timeout -k 10 120 python3 bench.py --workload c2 --steps 300 --warmup 20 > gpurun_out/${TAG}_c2_w${W}_$R.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_w${W}_$R.json')); print('c2 w$W', round(d['value']*1e3,4), 'ms', d['result'][:2])"
PGM_WG_CHAIN_BLOCKS=$W timeout -k 10 300 python3 bench.py --workload c1 --steps 100 --warmup 5 > gpurun_out/${TAG}_c1_w${W}_$R.json 2> gpurun_out/${TAG}_c1.err || { tail -30 gpurun_out/${TAG}_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c1_w${W}_$R.json')); print('c1 w$W', round(d['value']*1e3,4), 'ms')"
done
done
