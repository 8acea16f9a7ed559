# two ranks sharing the one GPU (gloo for the host-side collectives): the N>1 bench path end to end
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 100 --warmup 5 --dist-backend gloo > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail -30 gpurun_out/bench_n2.err; exit 1; }
cat gpurun_out/bench_n2.json
