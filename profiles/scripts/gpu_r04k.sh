# round 4: C3 at the driver's 20 steps over the 96 resident batches — user-mode queue count (4 / 6 / 8) and
# the resident ring (started inside the window / resident before it), interleaved, two repeats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04k}
c3() {  # label args...
  local L=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-ring-roofline "$@" > gpurun_out/${TAG}_c3_${L}_$R.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_${L}_$R.json')); r=d['roofline']; print('c3 $L', round(d['value']/1e9,2), 'G frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), d['parity']['ok'])"
}
for R in 1 2; do
  c3 q4 --queues 4
  c3 q6 --queues 6
  c3 q8 --queues 8
  c3 ring --launch ring
  c3 ringpre --launch ring --ring-prestart
done
# specialised batch kernels (contraction-only / product-only batches, PGM_BATCH_SPECIALISE=0 for the generic
# k_batch): parity of the kernel / inference suites at the new default, then C2 / C1 / C4 A/B
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_inference_gpu.py \
  tests/test_factor_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
ab() {  # label workload env -- args
  local L=$1 W=$2 E=$3; shift 4
  env $E timeout -k 10 300 python bench.py --workload $W "$@" --no-cpu-baseline > gpurun_out/${TAG}_${W}_${L}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_${L}_$R.json')); v=d['value']; print('$W $L', round(v*1e3,4) if v < 1 else round(v), round(d.get('ms_per_step', 0) or 0, 3))"
}
for R in 1 2; do
  for W in c2 c1; do
    ab generic $W PGM_BATCH_SPECIALISE=0 -- --steps 200 --warmup 20
    ab spec $W PGM_NOTHING=1 -- --steps 200 --warmup 20
  done
  ab generic c4 PGM_BATCH_SPECIALISE=0 -- --rows 4000 --steps 20 --warmup 3
  ab spec c4 PGM_NOTHING=1 -- --rows 4000 --steps 20 --warmup 3
done
timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps.txt 2>&1 && grep -A12 "steps," gpurun_out/${TAG}_c2_steps.txt
