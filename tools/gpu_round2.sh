# full round evidence + the N=2 bench path rehearsed with two gloo ranks sharing the one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r01}
bash tools/gpu_round.sh $TAG || exit 1
timeout -k 10 300 python bench.py --workload c4 --rows 4000 --steps 10 --warmup 2 > gpurun_out/bench_c4_4000.json 2> gpurun_out/bench_c4_4000.err || { tail -20 gpurun_out/bench_c4_4000.err; exit 1; }
cat gpurun_out/bench_c4_4000.json
bash tools/gpu_dist_rehearsal.sh || exit 1
