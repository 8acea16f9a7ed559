# round 4: the chain's LDS mirror (PGM_CHAIN_MIRROR=1: intermediates a later chain level reads also stored in LDS
# and read from there, LDS-only level barriers when every such read is mirrored) — parity of the kernel /
# inference / factor suites with it on, then C2 / C1 A/B and a level trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r04x}
PGM_CHAIN_MIRROR=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_inference_gpu.py \
  tests/test_factor_gpu.py tests/test_markov.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
ab() {  # label workload env
  local L=$1 W=$2 E=$3
  env $E timeout -k 10 300 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_${W}_${L}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${L}_$R.json')); print('$W $L', round(d['value']*1e3,4), 'ms')"
}
for R in 1 2 3; do
  for W in c2 c1; do
    ab off $W PGM_NOTHING=1
    ab mirror $W PGM_CHAIN_MIRROR=1
  done
done
cd /tmp && export TMPDIR=/tmp
PGM_CHAIN_MIRROR=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/${TAG}_c2trace" -o t --output-format csv -- \
  python3 "$ROOT/tools/c2_level_trace.py" run 200 > "$ROOT/gpurun_out/${TAG}_c2trace.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/${TAG}_c2trace.log"; exit 1; }
cd "$ROOT"
python3 tools/c2_level_trace.py summarize gpurun_out/${TAG}_c2trace > gpurun_out/${TAG}_c2_levels.txt && tail -3 gpurun_out/${TAG}_c2_levels.txt
