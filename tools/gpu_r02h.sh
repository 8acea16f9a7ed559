set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
PGM_ROWS_JIT_STORE=wt PGM_DQ_ACQ=none PGM_DQ_REL=none timeout -k 10 300 python tools/dq_latency.py > gpurun_out/dq_latency.json 2> gpurun_out/dq_latency.err || { tail -30 gpurun_out/dq_latency.err; exit 1; }
cat gpurun_out/dq_latency.json
