set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/program_steps.py c4 1000 > gpurun_out/steps_c4_1000.txt 2>&1 || { tail -20 gpurun_out/steps_c4_1000.txt; exit 1; }
head -30 gpurun_out/steps_c4_1000.txt | cut -c1-180
