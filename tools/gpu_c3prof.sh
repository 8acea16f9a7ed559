set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; ROOT=$GRAFT_REPO_ROOT
timeout -k 10 120 python tools/rows_sweep.py --rows 100000 --reps 200 --variants lds_values > gpurun_out/rows_sweep.txt 2>&1; grep rows gpurun_out/rows_sweep.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_c3b -o trace --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --steps 200 --warmup 10 > $ROOT/gpurun_out/prof_c3b.json 2>/dev/null || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$ROOT/gpurun_out/prof_c3b/trace_kernel_stats.csv')): print(r['Name'][:40].ljust(40), r['Calls'], r['AverageNs'], r['MinNs'])
"
python3 - <<'PY'
import csv
rows=[r for r in csv.DictReader(open('/root/repo/gpurun_out/prof_c3b/trace_kernel_trace.csv')) if 'rows_affine' in r['Kernel_Name']]
st=[int(r['Start_Timestamp']) for r in rows]; en=[int(r['End_Timestamp']) for r in rows]
gaps=[st[i+1]-en[i] for i in range(len(st)-1)]
gaps.sort(); print('launch gaps ns p10/p50/p90', gaps[len(gaps)//10], gaps[len(gaps)//2], gaps[9*len(gaps)//10])
PY
