set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bp_api_profile.py > gpurun_out/bp_api_profile.txt 2>&1 || { tail -30 gpurun_out/bp_api_profile.txt; exit 1; }
head -60 gpurun_out/bp_api_profile.txt
