# round 3: flat-mode contraction reductions with loads issued ahead (C1 / C2 / C4): parity + rates
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r03ac}
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_inference_gpu.py tests/test_markov.py tests/test_compat_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 1 2; do
timeout -k 10 120 python3 bench.py --workload c2 --steps 300 --warmup 20 > gpurun_out/${TAG}_c2_$R.json 2> gpurun_out/${TAG}_c2.err || { tail -30 gpurun_out/${TAG}_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_$R.json')); print('c2', round(d['value']*1e3,4), 'ms', d['result'][:2])"
timeout -k 10 300 python3 bench.py --workload c1 --steps 100 --warmup 5 > gpurun_out/${TAG}_c1_$R.json 2> gpurun_out/${TAG}_c1.err || { tail -30 gpurun_out/${TAG}_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c1_$R.json')); print('c1', round(d['value']*1e3,4), 'ms')"
done
for R in 4000 1000; do
timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_$R.json')); print('c4 rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms')"
done
TOP=30 timeout -k 10 200 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps.txt 2>&1 && head -3 gpurun_out/${TAG}_c2_steps.txt | tail -2
