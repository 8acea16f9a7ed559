# k_gemm_f64 record: gemm_bench (kernel trace incl. VGPR/AGPR counts), SQ counters, FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/gemm_bench.py > gpurun_out/bm_gemm_bench.txt 2>&1 || { tail -20 gpurun_out/bm_gemm_bench.txt; exit 1; }
cat gpurun_out/bm_gemm_bench.txt | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/bm_trace" -o trace --output-format csv -- python3 "$ROOT/tools/gemm_bench.py" > "$ROOT/gpurun_out/bm_trace.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/bm_trace.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -d "$ROOT/gpurun_out/bm_pmc_sq" -o pmc --output-format csv -- python3 "$ROOT/tools/gemm_bench.py" > "$ROOT/gpurun_out/bm_pmc_sq.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/bm_pmc_sq.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$ROOT/gpurun_out/bm_pmc_fetch" -o pmc --output-format csv -- python3 "$ROOT/tools/gemm_bench.py" > "$ROOT/gpurun_out/bm_pmc_fetch.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/bm_pmc_fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$ROOT/gpurun_out/bm_pmc_write" -o pmc --output-format csv -- python3 "$ROOT/tools/gemm_bench.py" > "$ROOT/gpurun_out/bm_pmc_write.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/bm_pmc_write.log"; exit 1; }
echo done
