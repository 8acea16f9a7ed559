# r06b: (1) ONE rocprofv3 kernel trace of the C2 line on the AQL chain, doorbell split at the ring wrap
# (1,000 timed queries x 20 packets: the 4,096-slot ring wraps 5 times); (2) C3 A/B of the row kernel's
# workgroup (320 -> 157 blocks, 192 -> 261 blocks per 100 k-row launch), three interleaved repeats at the
# driver's settings, each line with its raw dispatch timestamps; (3) the unprofiled C2 line for comparison
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/c2prof" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c2 --steps 1000 --warmup 20 --no-cpu-baseline > "$ROOT/$O/c2_prof.json" 2> "$ROOT/$O/c2_prof.err" \
  || { echo rocprof c2 failed; grep -v '^    @' "$ROOT/$O/c2_prof.err" | tail -12; exit 1; }
cd "$ROOT"
python tools/c2_trace_span.py $O/c2prof/*kernel_trace.csv $O/c2_prof.json > $O/c2_trace_span.json || exit 1
cat $O/c2_trace_span.json
timeout -k 10 120 python bench.py --workload c2 --steps 1000 --warmup 20 --no-cpu-baseline > $O/c2_plain.json 2> $O/c2_plain.err || exit 1
python -c "import json; d=json.load(open('$O/c2_plain.json')); print('c2 unprofiled', d['value']*1e3, 'ms', d['parity']['ok'])"
for rep in 1 2 3; do
  for wg in 320 192; do
    PGM_ROWS_JIT_WG=$wg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-subconfigs --no-c5 --no-api-e2e \
      > $O/c3_wg${wg}_$rep.json 2> $O/c3_wg${wg}_$rep.err || { tail -20 $O/c3_wg${wg}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c3_wg${wg}_$rep.json')); r=d['roofline']; print('wg $wg rep $rep', round(d['value']/1e9,2), 'G frac', round(r['frac'],3), 'grid', r['grid'], 'ring', round(r['single_launch_ring']['frac'],3))"
  done
done
python tools/c3_span_check.py $O/c3_wg*_*.json > $O/c3_span_check.json; echo "span check rc $?"
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06b/c3_span_check.json"))
for k, v in sorted(d.items()):
    print(k.split("/")[-1], round(v["frac_recomputed"], 3), round(v["frac_line"], 3), v["frac_agrees_within_5pct"],
          "in-flight", round(v["mean_in_flight_over_span"], 2), "ramp", round(v.get("ramp_ms", 0) * 1e3, 2), "us tail", round(v.get("tail_ms", 0) * 1e3, 2), "us",
          "span/ring", round(v.get("span_over_ring", 0), 3))
PY
