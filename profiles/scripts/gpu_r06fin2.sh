# r06fin2: final round-6 checkpoint at HEAD: the whole GPU suite, smoke, the default bench line as the driver runs it
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06fin2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06fin2/bench_default.json"))
r = d["roofline"]
print("C3", round(d["value"] / 1e9, 2), "G frac", round(r["frac"], 3), "wall", round(r["frac_wall"], 3), "ring", round(r["single_launch_ring"]["frac"], 3),
      "api", round(d["api_e2e"]["value"] / 1e6, 1), "M", "cpu", round(d["cpu_baseline"]["value"]), d["parity"]["ok"], r["grid"])
for k in ("c1", "c2", "c4"):
    s = d.get(k, {})
    print(k, s.get("value"), s.get("unit"), "parity", (s.get("parity") or {}).get("ok"), "cpu", (s.get("cpu_baseline") or {}).get("value"), s.get("error", ""), s.get("bench_s"))
print("c4 two", (d.get("c4", {}).get("two_in_flight") or {}).get("value"), "c2 launches", d["c2"].get("launches_per_query"))
c = d["c5"]
print("c5 host", round(c["host"]["value"] / 1e9, 3), "map", round(c["host_map"]["value"] / 1e9, 2), "rccl", round(c["rccl"]["value"] / 1e9, 2))
PY
