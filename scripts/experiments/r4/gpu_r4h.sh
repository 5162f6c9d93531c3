# Round 4 session h: FFT lengths beyond the powers of two (fft_any.hip) --
# the new tests first, then the whole GPU suite.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_any_c_gpu.py -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_any_c.log 2>&1 || { tail -60 $OUT/pytest_any_c.log; exit 1; }
tail -3 $OUT/pytest_any_c.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
