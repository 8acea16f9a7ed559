# r05d: C4 schedule dump + per-step PMC at 4,000 rows; C5 rotating roofline vs a rocprofv3 kernel trace
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
ROWS=4000 timeout -k 10 300 python tools/c4_dump.py gpurun_out/r05d/c4dump > gpurun_out/r05d/c4dump.log 2>&1 || { tail -20 gpurun_out/r05d/c4dump.log; exit 1; }
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d "$ROOT/gpurun_out/r05d/pmc_$C" -o p --output-format csv -- \
    python3 "$ROOT/tools/c4_step_pmc.py" run "$ROOT/gpurun_out/r05d/pmc_meta.json" > "$ROOT/gpurun_out/r05d/pmc_$C.log" 2>&1 \
    || { echo "pmc $C failed"; tail -5 "$ROOT/gpurun_out/r05d/pmc_$C.log"; exit 1; }
done
python3 "$ROOT/tools/c4_step_pmc.py" summarize "$ROOT/gpurun_out/r05d/pmc_meta.json" "$ROOT/gpurun_out/r05d/pmc_FETCH_SIZE" \
    "$ROOT/gpurun_out/r05d/pmc_WRITE_SIZE" > "$ROOT/gpurun_out/r05d/pmc_summary.json" || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r05d/c5trace" -o t --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c5 --steps 20 --warmup 5 > "$ROOT/gpurun_out/r05d/c5_prof.json" 2> "$ROOT/gpurun_out/r05d/c5_prof.err" || { tail -5 "$ROOT/gpurun_out/r05d/c5_prof.err"; exit 1; }
cd "$ROOT"
python3 tools/c5_trace_check.py $(ls gpurun_out/r05d/c5trace/*/t_kernel_trace.csv gpurun_out/r05d/c5trace/t_kernel_trace.csv 2>/dev/null | head -1) gpurun_out/r05d/c5_prof.json > gpurun_out/r05d/c5_trace_check.json
cat gpurun_out/r05d/c5_trace_check.json
python3 -c "import json; d=json.load(open('gpurun_out/r05d/pmc_summary.json')); print({k: d[k] for k in d if k != 'top' and k != 'steps'})"
