# round 3: parity with product trees; C4 rate; C3 queue-profiling A/B (PGM_DQ_PROFILE)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03r}
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_markov.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for R in 4000 1000; do
timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_$R.json')); print('c4 rows $R', round(d['value']), round(d['ms_per_step'],3), 'ms', round(d['frac_of_8TBps'],3))"
done
for R in 1 2 3; do
for P in 1 0; do
PGM_DQ_PROFILE=$P timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e > gpurun_out/${TAG}_direct20_prof${P}_$R.json 2> gpurun_out/${TAG}_d.err || { tail -30 gpurun_out/${TAG}_d.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_direct20_prof${P}_$R.json')); r=d['roofline']; print('profile $P', round(d['value']/1e9,2), round(r['frac'],3), round(r['frac_wall'],3))"
done
done
