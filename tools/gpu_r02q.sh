set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/c2_layout.py > gpurun_out/c2_layout.txt 2> gpurun_out/c2_layout.err || { tail -30 gpurun_out/c2_layout.err; exit 1; }
cat gpurun_out/c2_layout.txt
timeout -k 10 200 python tools/program_steps.py c2 > gpurun_out/steps_c2.txt 2>&1 || { tail -20 gpurun_out/steps_c2.txt; exit 1; }
head -12 gpurun_out/steps_c2.txt | cut -c1-150
