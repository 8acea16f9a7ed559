# C3 over several user-mode queues with batch sets larger than the 256 MB MALL (row-permuted batches): 20 / 400 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
for cfg in "4 4" "8 4" "24 4" "32 4" "24 2" "24 3" "24 6" "32 8"; do set -- $cfg
for K in 20 400; do
$T 300 python bench.py --steps $K --warmup 5 --batches $1 --queues $2 --no-cpu-baseline > gpurun_out/be_c3_b$1_q$2_$K.json 2> gpurun_out/be_c3_b$1_q$2_$K.err || { tail -30 gpurun_out/be_c3_b$1_q$2_$K.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[1],round(d['value']/1e9,2),'G/s step',round(d['ms_per_step']*1e3,3),'us kern',round(r['kernel_ms']*1e3,3),'GB/s',round(r['achieved']),d['parity']['ok'])" gpurun_out/be_c3_b$1_q$2_$K.json
done; done
