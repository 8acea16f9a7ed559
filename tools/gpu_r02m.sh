set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/c1_profile.py > gpurun_out/c1_profile.txt 2> gpurun_out/c1_profile.err || { tail -30 gpurun_out/c1_profile.err; exit 1; }
head -60 gpurun_out/c1_profile.txt
