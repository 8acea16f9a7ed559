# r05ae: chain vs per-level under the AQL chain (C1 / C2), forced both ways and tuned
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05ae
export TMPDIR=/tmp
for i in 1 2; do for F in tuned chain flat; do
  PGM_CHAIN_FORCE=$F timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05ae/c2_${F}_$i.json 2> gpurun_out/r05ae/c2.err || { tail -20 gpurun_out/r05ae/c2.err; exit 1; }
  PGM_CHAIN_FORCE=$F timeout -k 10 300 python -u bench.py --workload c1 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r05ae/c1_${F}_$i.json 2> gpurun_out/r05ae/c1.err || { tail -20 gpurun_out/r05ae/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05ae/c2_${F}_$i.json')); e=json.load(open('gpurun_out/r05ae/c1_${F}_$i.json')); print('$F c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
done; done
