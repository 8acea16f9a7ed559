# r06l: the bench line's api_e2e (why 83 M in the line vs 109 M alone): each call's time in the default line,
# and with the CPU baseline pool (forked before the GPU) left out
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-subconfigs --no-c5 > $O/a.json 2> $O/a.err || { tail -20 $O/a.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-subconfigs --no-c5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "
import json
for k in 'ab':
    d=json.load(open('$O/'+k+'.json'))['api_e2e']; print(k, round(d['value']/1e6,1), round(d['median_rows_per_s']/1e6,1), [round(x*1e3,3) for x in d['seconds_each']])"
timeout -k 10 120 python tools/e2e_stages.py 100000 20 > $O/e2e.txt 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
head -6 $O/e2e.txt
