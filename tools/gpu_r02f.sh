# does HIP overlap back-to-back kernels of one stream? kernel-trace gaps of the HIP launch; direct queue with/without barrier bit
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
P='import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d["value"]/1e9,2),"G rows/s",round(d["ms_per_step"]*1e3,3),"us/step kern",round(d["roofline"]["kernel_ms"]*1e3,3),"us parity",d["parity"]["ok"])'
G='
import csv,sys,statistics
rows=[r for r in csv.DictReader(open(sys.argv[1])) if "pgm_rows_jit" in r["Kernel_Name"]]
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
d=[int(r["End_Timestamp"])-int(r["Start_Timestamp"]) for r in rows]
g=[int(rows[i+1]["Start_Timestamp"])-int(rows[i]["End_Timestamp"]) for i in range(len(rows)-1)]
print(sys.argv[1],"n",len(rows),"dur med",statistics.median(d),"gap med",statistics.median(g),"gap min",min(g),"neg gaps",sum(x<0 for x in g))'
for L in hip direct; do
cd /tmp && PGM_ROWS_JIT_STORE=wt PGM_DQ_ACQ=none PGM_DQ_REL=none timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_$L -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 5 --no-cpu-baseline --launch $L > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/tr_$L.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/tr_$L.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "$G" gpurun_out/tr_$L/tr_kernel_trace.csv
done
for B in 1 0; do
PGM_ROWS_JIT_STORE=wt PGM_DQ_ACQ=none PGM_DQ_REL=none PGM_DQ_BARRIER=$B timeout -k 10 300 python bench.py --steps 400 --warmup 5 --no-cpu-baseline > gpurun_out/bar_$B.json 2> gpurun_out/bar_$B.err || { tail -30 gpurun_out/bar_$B.err; exit 1; }
python -c "$P" gpurun_out/bar_$B.json
done
