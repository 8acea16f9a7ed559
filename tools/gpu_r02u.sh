set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for V in "PGM_MARG_JX=-1" "PGM_MARG_JX=1" "PGM_MARG_JX=4" "PGM_MARG_JX=0" "PGM_MARG_BLOCKS=8192" "PGM_MARG_BLOCKS=512"; do
env $V timeout -k 10 300 python bench.py --workload c4 --rows 4000 --steps 10 --warmup 2 > gpurun_out/c4v.json 2> gpurun_out/c4v.err || { tail -30 gpurun_out/c4v.err; exit 1; }
python -c "import json,sys;d=json.load(open('gpurun_out/c4v.json'));print(sys.argv[1], round(d['value']), round(d['ms_per_step'],3))" "$V"
done
