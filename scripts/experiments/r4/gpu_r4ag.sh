# Round 4 session ag: the any-C and parity GPU tests on the library with the
# non-temporal IQ loads, and a bench line at C = 1536.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4ag; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_any_c_gpu.py tests/test_gpu_parity.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --R 64 --C 1536 --frames 400 \
  > $OUT/bench_c1536.json 2> $OUT/bench_c1536.err || { tail $OUT/bench_c1536.err; exit 1; }
cut -c 1-160 $OUT/bench_c1536.json
