# round 3: C4 per-step kernel durations, kept-order A/B (PGM_PM_KREV 0/1), plus FETCH per step for both
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03v}
for K in 0 1; do
PGM_PM_KREV=$K timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_kt$K -o k --output-format csv -- python3 tools/c4_step_pmc.py run gpurun_out/${TAG}_meta$K.json > gpurun_out/${TAG}_kt$K.log 2>&1 || { tail -30 gpurun_out/${TAG}_kt$K.log; exit 1; }
PGM_PM_KREV=$K timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_f$K -o f --output-format csv -- python3 tools/c4_step_pmc.py run gpurun_out/${TAG}_metaf$K.json > gpurun_out/${TAG}_f$K.log 2>&1 || { tail -30 gpurun_out/${TAG}_f$K.log; exit 1; }
done
python3 tools/c4_step_times.py gpurun_out/${TAG}_meta0.json krev0=gpurun_out/${TAG}_kt0 krev1=gpurun_out/${TAG}_kt1 > gpurun_out/${TAG}_steps.json
python3 - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_steps.json"))
print(d["total_us"])
for s in d["per_step"]:
    print(s["i"], s["level"], s["krev0"], s["krev1"], round(s["MB"] or 0, 1), s["note"][:60])
PY
