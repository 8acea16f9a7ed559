# r05ad: rocprofv3 kernel traces of the C2 and C4 lines (kernel-level evidence for DESIGN)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05ad
O=gpurun_out/r05ad
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d "$ROOT/$O/envcheck" -o t --output-format csv -- \
  python3 -c "import os; print('ROCPROF env:', sorted(k for k in os.environ if k.startswith('ROCPROF'))[:8])" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/c2" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c2 --steps 200 --warmup 20 > "$ROOT/$O/c2.json" 2> "$ROOT/$O/c2.err" || { tail -20 "$ROOT/$O/c2.err"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/c4" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c4 --rows 4000 --steps 20 --warmup 3 > "$ROOT/$O/c4.json" 2> "$ROOT/$O/c4.err" || { tail -20 "$ROOT/$O/c4.err"; exit 1; }
cd "$ROOT"
head -12 $O/c2/*kernel_stats.csv
head -12 $O/c4/*kernel_stats.csv
python -c "import json; d=json.load(open('$O/c2.json')); e=json.load(open('$O/c4.json')); print('c2 (profiled)', round(d['value']*1e3,4), 'ms; c4 (profiled)', round(e['value']/1e6,4), 'M/s')"
