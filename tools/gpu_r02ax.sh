set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u bench.py --workload c5 --c5-output map --steps 20 --warmup 5 > gpurun_out/c5_map.json 2> gpurun_out/c5_map.err || { tail -30 gpurun_out/c5_map.err; exit 1; }
cat gpurun_out/c5_map.json
$T 300 python -u bench.py --workload c5 --steps 20 --warmup 5 > gpurun_out/c5_marg.json 2> gpurun_out/c5_marg.err || { tail -30 gpurun_out/c5_marg.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/c5_marg.json').read().strip().splitlines()[-1]); print(d['value'], d['parity'])"
$T 300 python -u bench.py --workload c5 --c5-output map --gpus 2 --steps 20 --warmup 5 > gpurun_out/c5_map_n2.json 2> gpurun_out/c5_map_n2.err || { tail -30 gpurun_out/c5_map_n2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/c5_map_n2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['parity'], d.get('gather_ms'))"
