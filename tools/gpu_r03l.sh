# round 3: C4 per-step PMC (FETCH_SIZE / WRITE_SIZE separate passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03l}
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_c4pmc_fetch -o f --output-format csv -- python3 tools/c4_step_pmc.py run gpurun_out/${TAG}_c4_steps.json > gpurun_out/${TAG}_pmc_f.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_f.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_c4pmc_write -o w --output-format csv -- python3 tools/c4_step_pmc.py run gpurun_out/${TAG}_c4_steps.json > gpurun_out/${TAG}_pmc_w.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_w.log; exit 1; }
python3 tools/c4_step_pmc.py summarize gpurun_out/${TAG}_c4_steps.json gpurun_out/${TAG}_c4pmc_fetch gpurun_out/${TAG}_c4pmc_write > gpurun_out/${TAG}_c4_step_pmc.json && head -c 3500 gpurun_out/${TAG}_c4_step_pmc.json
