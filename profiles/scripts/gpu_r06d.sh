# r06d: the public API's new direct path (host pool scan + LUT map, device work first): its GPU tests,
# then the stage profile and the bench line's api_e2e measure
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_inference_gpu.py -k "predict or frame or wide or stochastic" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python tools/e2e_stages.py 100000 20 > $O/e2e_stages.txt 2> $O/e2e_stages.err || { tail -20 $O/e2e_stages.err; exit 1; }
head -24 $O/e2e_stages.txt
