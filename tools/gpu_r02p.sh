set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py -k "edits or c2 or threads" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_p.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_p.log; exit 1; }
tail -1 gpurun_out/pytest_p.log
timeout -k 10 300 python tools/c2_profile.py > gpurun_out/c2_profile.txt 2> gpurun_out/c2_profile.err || { tail -30 gpurun_out/c2_profile.err; exit 1; }
head -3 gpurun_out/c2_profile.txt
timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/n2.json 2> gpurun_out/n2.err || { tail -30 gpurun_out/n2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/n2.json'));print(d['n_gpus'],d['value'])"
