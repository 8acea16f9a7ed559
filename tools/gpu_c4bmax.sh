# level-batch size threshold for n-ary products (PGM_PRODN_BATCH_MAX) with the 16-B pair forms
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for R in 1000 4000; do
  for B in 2097152 4194304 8388608 2097152; do
    PGM_PRODN_BATCH_MAX=$B timeout -k 10 200 python bench.py --workload c4 --rows $R --steps 10 --warmup 2 > gpurun_out/c4b.json 2> gpurun_out/c4b.err || { tail gpurun_out/c4b.err; exit 1; }
    echo "C4 R=$R BMAX=$B $(python -c "import json; d=json.load(open('gpurun_out/c4b.json')); print(round(d['value']), round(d['ms_per_step'],3), round(d['achieved_GBps']))")"
  done
done
