# r06av: one rocprofv3 kernel trace of the C2 line at HEAD (10 packets per query), its chain spans recomputed by
# tools/c2_trace_span.py, and the unprofiled line beside it
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06av; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/c2prof" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c2 --steps 1000 --warmup 20 --no-cpu-baseline > "$ROOT/$O/c2_prof.json" 2> "$ROOT/$O/c2_prof.err" \
  || { echo rocprof c2 failed; grep -v '^    @' "$ROOT/$O/c2_prof.err" | tail -12; exit 1; }
cd "$ROOT"
python tools/c2_trace_span.py $O/c2prof/*kernel_trace.csv $O/c2_prof.json > $O/c2_trace_span.json || exit 1
cat $O/c2_trace_span.json
timeout -k 10 120 python bench.py --workload c2 --steps 1000 --warmup 20 --no-cpu-baseline > $O/c2_plain.json 2> $O/c2_plain.err || exit 1
python -c "import json; d=json.load(open('$O/c2_plain.json')); print('unprofiled', d['value']*1e6, 'us', d['launches_per_query'])"
