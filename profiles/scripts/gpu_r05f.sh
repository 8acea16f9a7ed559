# r05f: A/B of direct child-message operands (PGM_BP_DIRECT_MAX 8 vs 4), per-part step times
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05f
export TMPDIR=/tmp
for X in 4 8; do
  PGM_BP_DIRECT_MAX=$X ROWS=4000 timeout -k 10 400 python tools/c4_dump.py gpurun_out/r05f/dump$X > gpurun_out/r05f/dump$X.log 2>&1 || { tail -20 gpurun_out/r05f/dump$X.log; exit 1; }
  tail -1 gpurun_out/r05f/dump$X.log
done
for i in 1 2; do for X in 4 8; do
  PGM_BP_DIRECT_MAX=$X timeout -k 10 300 python -u bench.py --workload c4 --rows 4000 --steps 20 --warmup 3 > gpurun_out/r05f/c4_${X}_$i.json 2> gpurun_out/r05f/c4.err || { tail -20 gpurun_out/r05f/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05f/c4_${X}_$i.json')); print($X, round(d['value']/1e6,4), 'M/s')"
done; done
