# PMC HBM traffic of the batched-BP kernels (C4, 1000 rows): separate FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $ROOT/gpurun_out/c4pmc_$C -o pmc --output-format csv -- \
    python3 $ROOT/bench.py --workload c4 --rows 1000 --steps 1 --warmup 0 > /dev/null 2> $ROOT/gpurun_out/c4pmc_$C.err || { tail $ROOT/gpurun_out/c4pmc_$C.err; exit 1; }
done
ls $ROOT/gpurun_out/c4pmc_FETCH_SIZE
