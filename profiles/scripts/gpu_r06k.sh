# r06k checkpoint (part 2): rocprofv3 kernel trace of the default line, the C4 PMC passes, the C4 1,000-row
# line, C5 alone, and two ranks sharing the one GPU (gloo plumbing rehearsal of --gpus 2, not a scaling number)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --workload c4 --rows 1000 --steps 20 --warmup 3 > $O/c4_1000.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4_1000.json')); print('c4 1000', round(d['value']/1e6,4), 'M/s; two in flight', round(d['two_in_flight']['value']/1e6,4), d['parity']['ok'])"
timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', round(d['value']/1e9,3), 'G rows/s; kernel frac', round(d['roofline']['frac'],3))"
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-api-e2e --no-ring-roofline > $O/c3_world2.json 2> $O/c3_world2.err \
  || { tail -20 $O/c3_world2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3_world2.json')); c=d['c5']; print('world2 (one GPU)', d['n_gpus'], round(d['value']/1e9,2), 'G', d['parity']['ok'], 'c5 host', round(c['host']['value']/1e9,3), 'G', c['host']['parity']['ok'], 'rccl', round(c['rccl']['value']/1e9,3), c['rccl']['parity']['ok'])"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/prof" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-api-e2e --no-c5 --no-subconfigs > "$ROOT/$O/prof.json" 2> "$ROOT/$O/prof.err" \
  || { echo "trace pass failed"; tail -20 "$ROOT/$O/prof.err"; exit 1; }
grep -h "pgm_rows_ring\|pgm_rows_jit2" "$ROOT"/$O/prof/*kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d "$ROOT/$O/c4pmc_$C" -o p --output-format csv -- \
    python3 "$ROOT/tools/c4_step_pmc.py" run "$ROOT/$O/c4pmc_meta.json" > "$ROOT/$O/c4pmc_$C.log" 2>&1 \
    || { echo "pmc $C failed"; tail -5 "$ROOT/$O/c4pmc_$C.log"; exit 1; }
done
cd "$ROOT"
python3 tools/c4_step_pmc.py summarize $O/c4pmc_meta.json $O/c4pmc_FETCH_SIZE $O/c4pmc_WRITE_SIZE > $O/c4pmc_summary.json
python3 -c "import json; d=json.load(open('$O/c4pmc_summary.json')); print('c4 pmc fetch GB', round(d['fetch_bytes_x2']/1e9,2), 'write GB', round(d['write_bytes']/1e9,2), 'vs floor', round(d['ratio_to_floor'],3))"
