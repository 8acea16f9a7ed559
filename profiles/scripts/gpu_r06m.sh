# r06m: the C4 4,000-row schedule at HEAD, each step replayed alone (tools/c4_dump.py)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06m; mkdir -p $O
export TMPDIR=/tmp
ROWS=4000 timeout -k 10 300 python -u tools/c4_dump.py $O/d4000 > $O/d4000.log 2>&1 || { tail -20 $O/d4000.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06m/d4000/steps.json"))
tot = 0
for s in d["steps"]:
    tot += s["us"]
    print(s["i"], s["level"], round(s["us"], 1), "us", round(s["MB"], 1), "MB", round(s["MB"] / s["us"] / 1e3, 2) if s["us"] else 0, "TB/s", s["note"][:70])
print("sum", round(tot, 1), {k: v for k, v in d.items() if k != "steps"})
PY
