# big-clique product / fused product+marginal rates (tools/prodn_probe.py) vs the fused kernel's block count
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for R in 1000 4000; do
  for B in 2048 8192 32768; do
    PGM_MARG_BLOCKS=$B timeout -k 10 120 python tools/prodn_probe.py $R > gpurun_out/probe_${R}_$B.txt 2>&1 || { tail -20 gpurun_out/probe_${R}_$B.txt; exit 1; }
    echo "R=$R blocks=$B"; grep case gpurun_out/probe_${R}_$B.txt
  done
done
