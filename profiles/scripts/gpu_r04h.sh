# round 4: C1 / C2 after the multi-lane flat contraction change, C5 host-delivery stream A/B, C4 at the
# r04 defaults (two repeats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04h}
for W in c2 c1; do
  for R in 1 2; do
    timeout -k 10 300 python bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_${W}_$R.json 2> gpurun_out/${TAG}_$W.err || { tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${W}_$R.json')); print('$W', round(d['value']*1e3,4), 'ms/query')"
  done
done
timeout -k 10 300 python tools/program_steps.py c2 > gpurun_out/${TAG}_c2_steps.txt 2>&1 && grep "steps," gpurun_out/${TAG}_c2_steps.txt
grep -E "^ +[0-9.]+ us" gpurun_out/${TAG}_c2_steps.txt | head -8
for MODE in separate same; do
  for OUT in map marginals; do
    PGM_HOST_DELIVERY=$MODE timeout -k 10 300 python bench.py --workload c5 --c5-output $OUT --steps 50 --warmup 5 > gpurun_out/${TAG}_c5_${MODE}_$OUT.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_c5_${MODE}_$OUT.json')); print('c5 $MODE $OUT', round(d['value']/1e9,3), 'G rows/s', 'ms/step', round(d['ms_per_step'],3), 'copy', round(d['copy_ms'],3), d['parity']['ok'])"
  done
done
for R in 1 2; do
  for ROWS in 4000 1000; do
    timeout -k 10 300 python bench.py --workload c4 --rows $ROWS --steps 20 --warmup 3 > gpurun_out/${TAG}_c4_${ROWS}_$R.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_${ROWS}_$R.json')); print('c4 $ROWS', round(d['value']), round(d['ms_per_step'],3), 'ms')"
  done
done
