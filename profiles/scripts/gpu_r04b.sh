# round 4: new GPU tests (hazards, direct API path, pinned shard runs), the e2e stage profile, then
# the C3 working-set experiment (profiles/scripts/gpu_r04a.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04b}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hazards_gpu.py \
  "tests/test_inference_gpu.py::test_munin_predict_direct_path_against_golden" \
  "tests/test_plan_gpu.py::test_rows_shard_run_pinned_chunks_against_golden" \
  "tests/test_plan_gpu.py::test_rows_shard_run_matches_run" \
  "tests/test_distributed.py::test_sharded_host_delivery_matches_golden" \
  "tests/test_plan_gpu.py::test_row_ring_matches_bound_launches" "tests/test_plan_gpu.py::test_row_ring_exits_without_posts" \
  "tests/test_inference_gpu.py::test_threads_share_one_variable_elimination" -s > gpurun_out/${TAG}_newtests.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_newtests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python tools/e2e_profile.py > gpurun_out/${TAG}_e2e_profile.json 2> gpurun_out/${TAG}_e2e_profile.err || { tail -20 gpurun_out/${TAG}_e2e_profile.err; exit 1; }
cat gpurun_out/${TAG}_e2e_profile.json
for OUT in marginals map; do
  timeout -k 10 300 python bench.py --workload c5 --c5-output $OUT --steps 20 --warmup 5 > gpurun_out/${TAG}_c5_host_$OUT.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c5_host_$OUT.json')); print('c5 host $OUT', round(d['value']/1e9,3), 'G rows/s', 'ms/step', round(d['ms_per_step'],3), 'kernel', round(d['kernel_ms'],4), 'copy', round(d['copy_ms'],3), 'GB/s', round(d['copy_GBps'],1), d['parity'])"
done
bash profiles/scripts/gpu_r04a.sh r04a
