# round 4: API / threads changes (per-thread streams, faster categorical ingestion) and the C3 launch-shape
# sweep in the HBM regime (96 resident batches, 5.1x the Infinity Cache)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04e}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_inference_gpu.py::test_threads_share_one_variable_elimination" \
  "tests/test_inference_gpu.py::test_repeated_single_queries_see_new_evidence" \
  "tests/test_inference_gpu.py::test_alarm_queries" "tests/test_inference_gpu.py::test_munin_c2_query" \
  "tests/test_inference_gpu.py::test_munin_predict_direct_path_against_golden" \
  "tests/test_inference_gpu.py::test_munin_predict_categorical_frame" \
  "tests/test_inference_gpu.py::test_categorical_frame_with_nan_and_bad_category" -s > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|threads x" gpurun_out/${TAG}_tests.log | tail -14
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python tools/e2e_profile.py > gpurun_out/${TAG}_e2e_profile.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 1; }
cat gpurun_out/${TAG}_e2e_profile.json
c3() {  # label args / env
  local L=$1; shift
  env $ENVS timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-ring-roofline "$@" > gpurun_out/${TAG}_c3_$L.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_$L.json')); r=d['roofline']; print('c3 $L', round(d['value']/1e9,2), 'G', 'ms/step', round(d['ms_per_step']*1e3,2), 'us', 'frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), 'grid', r.get('grid'))"
}
ENVS=PGM_NOTHING=1 c3 q4_wg512
ENVS=PGM_NOTHING=1 c3 q2_wg512 --queues 2
ENVS=PGM_NOTHING=1 c3 q8_wg512 --queues 8
ENVS=PGM_ROWS_JIT_WG=256 c3 q4_wg256
ENVS=PGM_ROWS_JIT_WG=1024 c3 q4_wg1024
ENVS=PGM_ROWS_JIT_WG=128 c3 q4_wg128
ENVS=PGM_ROWS_JIT_WG=192 c3 q4_wg192
ENVS=PGM_ROWS_JIT_WG=256 c3 q8_wg256 --queues 8
ENVS=PGM_NOTHING=1 c3 ring_prestart --launch ring --ring-prestart
ENVS=PGM_NOTHING=1 c3 ring --launch ring
ENVS=PGM_NOTHING=1 c3 q4_wg512_400 --steps 400
ENVS=PGM_NOTHING=1 c3 ring_prestart_400 --launch ring --ring-prestart --steps 400
