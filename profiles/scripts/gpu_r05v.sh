# r05v: C1 direct chain vs graph, 200 and 300 steps (the checkpoint's C1 figure was 0.10 ms)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05v
export TMPDIR=/tmp
for i in 1 2; do for S in 300 200; do for X in 1 0; do
  PGM_QUERY_DIRECT=$X timeout -k 10 300 python -u bench.py --workload c1 --steps $S --warmup 30 --no-cpu-baseline > gpurun_out/r05v/c1_${X}_${S}_$i.json 2> gpurun_out/r05v/c1.err || { tail -20 gpurun_out/r05v/c1.err; exit 1; }
  python -c "import json; e=json.load(open('gpurun_out/r05v/c1_${X}_${S}_$i.json')); print('direct=$X steps=$S c1', round(e['value']*1e3,4), 'ms/query')"
done; done; done
