# C4: row pairs per lane in the specialised steps (forced XI, or a per-step minimum) at 1,000 / 4,000 rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P='import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.4f" % d["ms_per_step"], "exec_GBps=%.0f" % d.get("executed_step_GBps", 0))'
for rows in 4000 1000; do
for cfg in base PGM_PM_XI=2 PGM_PM_XI_MIN=2 PGM_PM_XI=4 PGM_PM_XI_MIN=4 base PGM_PM_XI=2 PGM_PM_XI_MIN=2; do
  E=""; [ $cfg != base ] && E=$cfg
  T=$(echo $cfg | tr '=' '_')_${rows}_$RANDOM
  env $E timeout -k 10 200 python bench.py --workload c4 --rows $rows --steps 20 --warmup 3 > gpurun_out/c4x_$T.json 2> gpurun_out/c4x_$T.err || { tail -20 gpurun_out/c4x_$T.err; exit 1; }
  python -c "$P" gpurun_out/c4x_$T.json "$cfg rows=$rows"
done
done
