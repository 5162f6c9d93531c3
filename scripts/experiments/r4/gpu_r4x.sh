# Round 4 session x: edge shapes of the non-power-of-two receivers.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4x; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_any_c_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_any_c.log 2>&1 || { tail -60 $OUT/pytest_any_c.log; exit 1; }
tail -2 $OUT/pytest_any_c.log
