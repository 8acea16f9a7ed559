set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/c2_profile.py > gpurun_out/c2_profile.txt 2> gpurun_out/c2_profile.err || { tail -30 gpurun_out/c2_profile.err; exit 1; }
head -3 gpurun_out/c2_profile.txt
timeout -k 10 300 python bench.py --workload c2 --steps 20 --warmup 2 > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -30 gpurun_out/c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c2.json'));print({k:v for k,v in d.items() if k!='result'})"
timeout -k 10 300 python bench.py --workload c1 --steps 100 --warmup 2 > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail -30 gpurun_out/c1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c1.json'));print(d)"
