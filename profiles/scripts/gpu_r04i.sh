# round 4: C5 host delivery on two stream lanes (HostDelivery mode "lanes", the new default) against one stream
# ("same"), MAP and marginals; the sharded host-delivery parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04i}
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_distributed.py -k host_delivery > gpurun_out/${TAG}_dist.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_dist.log; exit 1; }
tail -2 gpurun_out/${TAG}_dist.log
for R in 1 2; do
  for MODE in lanes same; do
    for OUT in map marginals; do
      PGM_HOST_DELIVERY=$MODE timeout -k 10 300 python bench.py --workload c5 --c5-output $OUT --steps 50 --warmup 5 > gpurun_out/${TAG}_c5_${MODE}_${OUT}_$R.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/${TAG}_c5_${MODE}_${OUT}_$R.json')); print('c5 $MODE $OUT', round(d['value']/1e9,3), 'G rows/s', 'ms/step', round(d['ms_per_step'],3), 'kernel', round(d['kernel_ms'],4), 'copy', round(d['copy_ms'],3), d['parity']['ok'])"
    done
  done
done
