# round 3: normalisation in two batched launches (C1 / C2); inference parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_markov.py tests/test_plan_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 1 2; do
timeout -k 10 120 python3 bench.py --workload c2 --steps 300 --warmup 20 > gpurun_out/${TAG}_c2_$R.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_$R.json')); print('c2', round(d['value']*1e3,4), 'ms', d['result'][:2])"
timeout -k 10 300 python3 bench.py --workload c1 --steps 100 --warmup 5 > gpurun_out/${TAG}_c1_$R.json 2> gpurun_out/${TAG}_c1.err || { tail -30 gpurun_out/${TAG}_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c1_$R.json')); print('c1', round(d['value']*1e3,4), 'ms')"
done
