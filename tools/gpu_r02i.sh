# write-through stores + direct queue defaults: GPU suite, smoke, C3 (20/400 steps, direct and hip), C5, rocprof + PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
P='import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d["value"]/1e9,2),"G rows/s",round(d["ms_per_step"]*1e3,3),"us/step kern",round(d["roofline"]["kernel_ms"]*1e3,3),"us parity",d["parity"]["ok"])'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for L in direct hip; do for K in 20 400; do
timeout -k 10 300 python bench.py --steps $K --warmup 5 --no-cpu-baseline --launch $L > gpurun_out/c3_${L}_$K.json 2> gpurun_out/c3_${L}_$K.err || { tail -30 gpurun_out/c3_${L}_$K.err; exit 1; }
python -c "$P" gpurun_out/c3_${L}_$K.json
done; done
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > gpurun_out/c5_n1.json 2> gpurun_out/c5_n1.err || { tail -30 gpurun_out/c5_n1.err; exit 1; }
python -c "$P" gpurun_out/c5_n1.json
bash tools/gpu_profile.sh r02i --steps 200 --warmup 10 || exit 1
