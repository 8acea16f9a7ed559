# r05an: the chain's first packet acquiring at agent scope instead of system (codes live in coherent host memory)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; mkdir -p gpurun_out/r05an
export TMPDIR=/tmp
PGM_DQ_FIRST_ACQ=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_inference_gpu.py -k "direct_chain or munin_c2 or alarm" > gpurun_out/r05an/t0.log 2>&1 || { tail -30 gpurun_out/r05an/t0.log; exit 1; }
tail -1 gpurun_out/r05an/t0.log
for i in 1 2; do for A in 2 1; do
  PGM_DQ_FIRST_ACQ=$A timeout -k 10 300 python -u bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05an/c2_${A}_$i.json 2> gpurun_out/r05an/c2.err || { tail -20 gpurun_out/r05an/c2.err; exit 1; }
  PGM_DQ_FIRST_ACQ=$A timeout -k 10 300 python -u bench.py --workload c1 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r05an/c1_${A}_$i.json 2> gpurun_out/r05an/c1.err || { tail -20 gpurun_out/r05an/c1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05an/c2_${A}_$i.json')); e=json.load(open('gpurun_out/r05an/c1_${A}_$i.json')); print('first_acq=$A c2', round(d['value']*1e3,4), 'c1', round(e['value']*1e3,4), 'ms/query', d['parity']['ok'])"
done; done
