set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/c2_profile.py > gpurun_out/c2_profile.txt 2> gpurun_out/c2_profile.err || { tail -30 gpurun_out/c2_profile.err; exit 1; }
head -45 gpurun_out/c2_profile.txt
timeout -k 10 200 python tools/program_steps.py c2 > gpurun_out/steps_c2.txt 2>&1; grep -E "steps|gemm" gpurun_out/steps_c2.txt | head -8 | cut -c1-160
