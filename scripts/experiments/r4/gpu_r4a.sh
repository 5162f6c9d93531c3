# Round 4 first GPU session: new launcher/split tests, then the default bench
# line with the timed-output check.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_antenna_split_gpu.py > $OUT/pytest_split.log 2>&1 || { tail -30 $OUT/pytest_split.log; exit 1; }
tail -3 $OUT/pytest_split.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
