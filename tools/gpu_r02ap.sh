set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c4_single.py > gpurun_out/c4_single.json 2> gpurun_out/c4_single.err || { tail -30 gpurun_out/c4_single.err; exit 1; }
cat gpurun_out/c4_single.json
