# round 4: C3 workgroup-size confirmation in the HBM regime (96 batches, 4 queues; three interleaved
# repeats) and the direct API path's stage profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04f}
timeout -k 10 300 python tools/e2e_profile.py > gpurun_out/${TAG}_e2e_profile.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_e2e_profile.json')); print({k: v for k, v in d.items() if k != 'cprofile_predict_probability_x5'}); print('\n'.join(d['cprofile_predict_probability_x5']))"
c3() {  # label wg
  env PGM_ROWS_JIT_WG=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-ring-roofline > gpurun_out/${TAG}_c3_$1.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_$1.json')); r=d['roofline']; print('c3 $1', round(d['value']/1e9,2), 'G', 'frac', round(r['frac'],3), 'wall', round(r['frac_wall'],3), r['grid'])"
}
for R in 1 2 3; do
  for WG in 192 512 128 1024 320; do
    c3 wg${WG}_$R $WG
  done
done
for OUT in map marginals; do
  timeout -k 10 300 python bench.py --workload c5 --c5-output $OUT --steps 50 --warmup 5 > gpurun_out/${TAG}_c5_host_$OUT.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c5_host_$OUT.json')); print('c5 host $OUT', round(d['value']/1e9,3), 'G rows/s', 'ms/step', round(d['ms_per_step'],3), 'kernel', round(d['kernel_ms'],4), 'copy', round(d['copy_ms'],3), 'GB/s', round(d['copy_GBps'],1))"
done
