set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for V in "PGM_ROWS_JIT_WG=256" "PGM_ROWS_JIT_WG=128" "PGM_ROWS_JIT_WG=64" "PGM_JIT2_MIN_ROWS=1" "PGM_JIT2_MIN_ROWS=1 PGM_ROWS_JIT_WG=128" "PGM_JIT2_MIN_ROWS=1 PGM_ROWS_JIT_WG=64"; do
env $V timeout -k 10 300 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/c3v.json 2> gpurun_out/c3v.err || { tail -30 gpurun_out/c3v.err; exit 1; }
python -c "import json,sys;d=json.load(open('gpurun_out/c3v.json'));print(sys.argv[1], round(d['value']/1e9,2), round(d['ms_per_step']*1e3,3), round(d['roofline']['kernel_ms']*1e3,3), d['parity']['ok'])" "$V"
done
