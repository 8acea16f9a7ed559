set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; ROOT=$GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/floor 100000 > gpurun_out/floor_100k.txt 2>&1 && grep -v "shape\|env\|store " gpurun_out/floor_100k.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_floor3 -o trace --output-format csv -- $ROOT/tools/floor 100000 > /dev/null 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$ROOT/gpurun_out/prof_floor3/trace_kernel_stats.csv')): print(r['Name'][:40].ljust(40), r['Calls'], r['AverageNs'], r['MinNs'])
"
