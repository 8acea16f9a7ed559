# r06a: GPU suite, smoke, the default bench line (driver args) with its c1/c2/c4 sub-objects, then ONE
# rocprofv3 kernel trace of the C2 line on the AQL chain (query queue profiling left on; no bypass)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo pytest failed; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 360 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err \
  || { tail -30 $O/bench_default.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06a/bench_default.json"))
print("C3", round(d["value"] / 1e9, 2), "G rows/s frac", round(d["roofline"]["frac"], 3), "wall", round(d["roofline"]["frac_wall"], 3))
for k in ("c1", "c2", "c4"):
    s = d.get(k, {})
    print(k, s.get("value"), s.get("unit"), "parity", (s.get("parity") or {}).get("ok"), "cpu", (s.get("cpu_baseline") or {}).get("value"), s.get("error", ""), s.get("bench_s"))
print("c4 two", (d.get("c4", {}).get("two_in_flight") or {}).get("value"))
PY
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/c2prof" -o trace --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c2 --steps 200 --warmup 20 --no-cpu-baseline > "$ROOT/$O/c2_prof.json" 2> "$ROOT/$O/c2_prof.err" \
  || { echo rocprof c2 failed; tail -30 "$ROOT/$O/c2_prof.err"; exit 1; }
cd "$ROOT"
head -8 $O/c2prof/*kernel_stats.csv
python -c "import json; d=json.load(open('$O/c2_prof.json')); print('c2 under rocprofv3', d['value']*1e3, 'ms', d['dispatch'], d['parity']['ok'])"
