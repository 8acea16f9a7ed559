# round 4: C2 / C1 with the tail of the contraction path as one single-workgroup launch (PGM_WG_CHAIN_BLOCKS
# 4 / 8) whose contraction descriptors are staged in LDS (k_batch_wg_c; PGM_CHAIN_LDS=0: the r03 k_batch_wg),
# against one launch per level (0, the default); kernel / inference parity with chains on; a level trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04n}
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "level_chain or batch" > gpurun_out/${TAG}_chain_test.log 2>&1 || { tail -30 gpurun_out/${TAG}_chain_test.log; exit 1; }
tail -1 gpurun_out/${TAG}_chain_test.log
PGM_WG_CHAIN_BLOCKS=8 timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_inference_gpu.py \
  -k "c2 or alarm or query or bn6" > gpurun_out/${TAG}_inf_chain8.log 2>&1 || { tail -30 gpurun_out/${TAG}_inf_chain8.log; exit 1; }
tail -1 gpurun_out/${TAG}_inf_chain8.log
ab() {  # label workload env...
  local L=$1 W=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_${W}_${L}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${L}_$R.json')); print('$W $L', round(d['value']*1e3,4), 'ms')"
}
for R in 1 2; do
  for W in c2 c1; do
    ab off $W PGM_WG_CHAIN_BLOCKS=0
    ab chain4 $W PGM_WG_CHAIN_BLOCKS=4
    ab chain8 $W PGM_WG_CHAIN_BLOCKS=8
    ab chain8gen $W PGM_WG_CHAIN_BLOCKS=8 PGM_CHAIN_LDS=0
  done
done
cd /tmp && export TMPDIR=/tmp
PGM_WG_CHAIN_BLOCKS=8 timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/${TAG}_c2trace" -o t --output-format csv -- \
  python3 "$ROOT/tools/c2_level_trace.py" run 200 > "$ROOT/gpurun_out/${TAG}_c2trace.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/${TAG}_c2trace.log"; exit 1; }
cd "$ROOT"
python3 tools/c2_level_trace.py summarize gpurun_out/${TAG}_c2trace > gpurun_out/${TAG}_c2_levels.txt && tail -14 gpurun_out/${TAG}_c2_levels.txt
