# r06aq: where the kept-dim reorder (PGM_NARY_KORDER=1) breaks C2's fused program: every float64 buffer the
# program keeps, after one run, with and without it
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06aq; mkdir -p $O
export TMPDIR=/tmp
PGM_NARY_KORDER=0 timeout -k 10 300 python -u tools/korder_diff.py $O/k0.npz > $O/k0.txt 2>&1 || { tail -20 $O/k0.txt; exit 1; }
PGM_NARY_KORDER=1 timeout -k 10 300 python -u tools/korder_diff.py $O/k1.npz > $O/k1.txt 2>&1 || { tail -20 $O/k1.txt; exit 1; }
tail -1 $O/k0.txt | cut -c1-300; tail -1 $O/k1.txt | cut -c1-300
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/r06aq/k0.npz"); b = np.load("gpurun_out/r06aq/k1.npz")
bad = 0
for i, kname in enumerate(a.files):
    x, y = a[kname], b[kname]
    if x.shape != y.shape:
        print(i, "shape", x.shape, y.shape); bad += 1; continue
    d = np.max(np.abs(x - y) / (np.abs(x) + 1e-300)) if x.size else 0
    if not np.isfinite(d) or d > 1e-9:
        print(i, x.shape, "rel diff", d, "nan", np.isnan(y).sum(), x[:4], y[:4]); bad += 1
        if bad > 8: break
print("tensors", len(a.files), "differing", bad)
PY
