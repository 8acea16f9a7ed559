# C4 at 1,000 rows: specialised-step thresholds and level-batch sizes re-checked at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.4f" % d["ms_per_step"])'
for cfg in base PGM_PM_JIT_MIN=65536 PGM_PM_JIT_MIN=131072 PGM_PM_PREFER_MIN=65536 PGM_PM_PREFER_MIN=131072 "PGM_PM_JIT_MIN=65536 PGM_PM_PREFER_MIN=65536" PGM_PRODN_BATCH_MAX=524288 PGM_PRODN_BATCH_MAX=8388608 base; do
  E=""; [ "$cfg" != base ] && E=$cfg
  T=$(echo $cfg | tr ' =' '__')_$RANDOM
  env $E timeout -k 10 200 python bench.py --workload c4 --rows 1000 --steps 20 --warmup 3 > gpurun_out/c4s_$T.json 2> gpurun_out/c4s_$T.err || { tail -20 gpurun_out/c4s_$T.err; exit 1; }
  python -c "$P" gpurun_out/c4s_$T.json "$cfg"
done
