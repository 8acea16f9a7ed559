# round 4: host-side profile of the C2 query path on the GPU box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r04q}
timeout -k 10 300 python tools/c2_host_profile.py 2000 > gpurun_out/${TAG}_c2_host.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c2_host.txt; exit 1; }
grep -v "^Extension" gpurun_out/${TAG}_c2_host.txt | head -50
