# r06ap: the N > 1 path at HEAD rehearsed on the one GPU (bench.py --gpus 2: two ranks share the card)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06ap; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-api-e2e --no-ring-roofline > $O/c3_world2.json 2> $O/c3_world2.err \
  || { tail -20 $O/c3_world2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3_world2.json')); c=d['c5']; print('world2 (one GPU)', d['n_gpus'], round(d['value']/1e9,2), 'G', d['parity']['ok'], 'c5 host', round(c['host']['value']/1e9,3), 'G', c['host']['parity']['ok'], 'rccl', round(c['rccl']['value']/1e9,3), c['rccl']['parity']['ok'])"
