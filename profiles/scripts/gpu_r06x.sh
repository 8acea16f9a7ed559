# r06x: C4 (4,000 rows, one batch at a time) under a rocprofv3 kernel trace: per launch of the sweep, kernel
# time and the gap before it (tools/c4_sweep_gaps.py)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06x; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o c4 -- python3 $ROOT/bench.py --workload c4 --rows 4000 --steps 20 --warmup 3 --c4-inflight 1 --no-cpu-baseline > $ROOT/$O/c4_prof.json 2> $ROOT/$O/prof.err || { tail -30 $ROOT/$O/prof.err; exit 1; }
cd $ROOT
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/c4_sweep_gaps.py $T > $O/gaps.json && python -c "
import json; d=json.load(open('$O/gaps.json'))
print('period', d['period'], 'sweeps', d['sweeps'], 'kernels', d['kernel_sum_us'], 'gaps', d['gap_sum_us'], 'span', d['sweep_span_us'])
for q in d['positions']: print(q['p'], q['us'], q['gap_before_us'], q['kernel'])"
gzip -c $T > $O/c4_kernel_trace.csv.gz
