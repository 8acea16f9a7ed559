# r05ab: C4 two in flight, lane 0 at high stream priority (A/B)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05ab
export TMPDIR=/tmp
for i in 1 2; do for P in 0 1; do for R in 4000 1000; do
  PGM_C4_LANE_PRIO=$P timeout -k 10 300 python -u bench.py --workload c4 --rows $R --steps 20 --warmup 3 > gpurun_out/r05ab/c4_${P}_${R}_$i.json 2> gpurun_out/r05ab/c4.err || { tail -20 gpurun_out/r05ab/c4.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05ab/c4_${P}_${R}_$i.json')); print('prio=$P', $R, round(d['value']/1e6,4), 'M/s one', round(d['one_in_flight']['value']/1e6,4), d['parity']['ok'])"
done; done; done
