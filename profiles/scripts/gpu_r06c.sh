# r06c: the new GPU tests (API extras, public calibrate_batch with lanes), then where C2's and the public
# API's time goes (tools/c2_split.py, tools/e2e_stages.py)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"; cd "$ROOT"; O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_factor_gpu.py::test_api_extras_against_reference tests/test_inference_gpu.py::test_calibrate_batch_public_api_inflight \
  tests/test_inference_gpu.py::test_munin_c2_root_mass > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python tools/c2_split.py 2000 > $O/c2_split.json 2> $O/c2_split.err || { tail -20 $O/c2_split.err; exit 1; }
cat $O/c2_split.json
timeout -k 10 200 python tools/e2e_stages.py 100000 20 > $O/e2e_stages.txt 2> $O/e2e_stages.err || { tail -20 $O/e2e_stages.err; exit 1; }
head -30 $O/e2e_stages.txt
