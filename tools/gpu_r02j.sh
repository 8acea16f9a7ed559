set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for F in system agent none; do
PGM_DQ_FRESH_ACQ=$F timeout -k 10 300 python tools/dq_latency.py > gpurun_out/dq_latency_$F.json 2> gpurun_out/dq_latency_$F.err || { tail -30 gpurun_out/dq_latency_$F.err; exit 1; }
echo $F; cat gpurun_out/dq_latency_$F.json
done
