# store form (plain / write-through) x direct-queue release scope, and the HIP launch; WRITE_SIZE per launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
P='import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d["value"]/1e9,2),"G rows/s",round(d["ms_per_step"]*1e3,3),"us/step kern",round(d["roofline"]["kernel_ms"]*1e3,3),"us parity",d["parity"]["ok"])'
for ST in plain wt; do
for R in none agent; do
PGM_ROWS_JIT_STORE=$ST PGM_DQ_REL=$R timeout -k 10 300 python bench.py --steps 400 --warmup 5 --no-cpu-baseline > gpurun_out/st_${ST}_$R.json 2> gpurun_out/st_${ST}_$R.err || { tail -30 gpurun_out/st_${ST}_$R.err; exit 1; }
python -c "$P" gpurun_out/st_${ST}_$R.json
done
PGM_ROWS_JIT_STORE=$ST timeout -k 10 300 python bench.py --steps 400 --warmup 5 --no-cpu-baseline --launch hip > gpurun_out/st_${ST}_hip.json 2> gpurun_out/st_${ST}_hip.err || { tail -30 gpurun_out/st_${ST}_hip.err; exit 1; }
python -c "$P" gpurun_out/st_${ST}_hip.json
done
cd /tmp
for ST in plain wt; do for R in none agent; do
PGM_ROWS_JIT_STORE=$ST PGM_DQ_REL=$R timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmcw_${ST}_$R -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/pmcw_${ST}_$R.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmcw_${ST}_$R.err; exit 1; }
python3 -c "
import csv,statistics,sys
v=[float(r['Counter_Value']) for r in csv.DictReader(open(sys.argv[1])) if 'pgm_rows_jit' in r['Kernel_Name']]
print(sys.argv[1], 'launches', len(v), 'WRITE_SIZE KB median', statistics.median(v) if v else None)" $GRAFT_REPO_ROOT/gpurun_out/pmcw_${ST}_$R/pmc_counter_collection.csv
done; done
