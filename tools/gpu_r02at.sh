# C3 at the driver's 20 steps: first-dispatch acquire scope A/B (three passes each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
run() { local lab=$1; shift
  env "$@" $T 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c3_$lab.json 2> gpurun_out/c3_$lab.err || { echo "$lab failed"; tail -20 gpurun_out/c3_$lab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c3_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,3), round(d['roofline']['kernel_ms']*1e3,3))"
}
for p in 1 2 3; do
run sys_$p
run agent_$p PGM_DQ_FRESH_ACQ=agent
run none_$p PGM_DQ_FRESH_ACQ=none
true
done
