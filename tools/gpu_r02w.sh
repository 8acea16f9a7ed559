set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py tests/test_kernels_gpu.py -k "bp or BP or calibrat or product_n or jt3" -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_w.log 2>&1 || { echo pytest failed; tail -60 gpurun_out/pytest_w.log; exit 1; }
tail -1 gpurun_out/pytest_w.log
for V in "PGM_MARG_KORDER=1" "PGM_MARG_KORDER=0"; do for R in 1000 4000; do
env $V timeout -k 10 300 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/c4v.json 2> gpurun_out/c4v.err || { tail -30 gpurun_out/c4v.err; exit 1; }
python -c "import json,sys;d=json.load(open('gpurun_out/c4v.json'));print(sys.argv[1], sys.argv[2], round(d['value']), round(d['ms_per_step'],3))" "$V" $R
done; done
