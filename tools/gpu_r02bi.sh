# C4: rows split into S independent calibration batches, each graph on its own stream
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
for cfg in "4000 1" "4000 2" "4000 4" "1000 1" "1000 2" "1000 4" "8000 2"; do set -- $cfg
$T 300 python bench.py --workload c4 --rows $1 --c4-streams $2 --steps 10 --warmup 2 > gpurun_out/bi_c4_$1_s$2.json 2> gpurun_out/bi_c4_$1_s$2.err || { tail -30 gpurun_out/bi_c4_$1_s$2.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']),'cal/s',round(d['ms_per_step'],3),'ms',round(d['frac_of_8TBps'],3))" gpurun_out/bi_c4_$1_s$2.json
done
