# C4 (pathfinder batched BP, 4,000 rows): specialised-step knobs re-checked at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.4f" % d["ms_per_step"], "GBps=%.0f" % d["achieved_GBps"], "exec_GBps=%.0f" % d.get("executed_step_GBps", 0))'
for cfg in base PGM_PM_UNROLL=4 PGM_PM_UNROLL=16 PGM_PM_XI=2 PGM_PM_NT=0 PGM_PM_XCD=0 PGM_PM_MNT=0 PGM_PM2_MAX_ACC=8 PGM_PM2_MAX_ACC=32 base; do
  E=""; [ $cfg != base ] && E=$cfg
  T=$(echo $cfg | tr '=' '_')_$RANDOM
  env $E timeout -k 10 200 python bench.py --workload c4 --rows 4000 --steps 10 --warmup 2 > gpurun_out/c4k_$T.json 2> gpurun_out/c4k_$T.err || { tail -20 gpurun_out/c4k_$T.err; exit 1; }
  python -c "$P" gpurun_out/c4k_$T.json $cfg
done
