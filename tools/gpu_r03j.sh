# round 3: single-query path with host-resident codes/result + depth-aware C2 path; inference suites
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03j}
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_inference_gpu.py -k "repeated_single or alarm_queries or bn6 or munin_c2" > gpurun_out/${TAG}_pytest_q.log 2>&1 || { echo query tests failed; tail -60 gpurun_out/${TAG}_pytest_q.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_q.log
timeout -k 10 300 python -u tools/c1_check.py > gpurun_out/${TAG}_c1_check.txt 2>&1 || { tail -8 gpurun_out/${TAG}_c1_check.txt; exit 1; }
timeout -k 10 300 python bench.py --workload c1 --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_c1.json 2> gpurun_out/${TAG}_bench_c1.err || { tail -30 gpurun_out/${TAG}_bench_c1.err; exit 1; }
timeout -k 10 300 python bench.py --workload c2 --steps 20 --warmup 2 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { tail -30 gpurun_out/${TAG}_bench_c2.err; exit 1; }
head -c 420 gpurun_out/${TAG}_bench_c1.json gpurun_out/${TAG}_bench_c2.json; echo
LEVELS=1 TOP=10 timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_levels.txt 2>&1 || { tail -30 gpurun_out/${TAG}_c2_levels.txt; exit 1; }
head -3 gpurun_out/${TAG}_c2_levels.txt
timeout -k 10 900 $T -m gpu tests/test_inference_gpu.py tests/test_markov.py tests/test_compat_gpu.py > gpurun_out/${TAG}_pytest_inf.log 2>&1 || { echo inference tests failed; tail -80 gpurun_out/${TAG}_pytest_inf.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_inf.log
