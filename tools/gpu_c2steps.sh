# C2 step-level view
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/program_steps.py c2 > gpurun_out/steps_c2.txt 2>&1; grep gemm gpurun_out/steps_c2.txt | head -8 | cut -c1-200
