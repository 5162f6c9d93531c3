# Round 4 session t: the C = 1536 receiver (frame_td1536.hip): any-C tests,
# the GPU suite, same-process A/B against the generic any-C kernel (variant
# "generic" = the library before it), and the bench line at R = 64.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_any_c_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_any_c.log 2>&1 || { tail -60 $OUT/pytest_any_c.log; exit 1; }
tail -2 $OUT/pytest_any_c.log
timeout -k 10 240 python scripts/abx.py --C 1536 --R 64 --frames 200 --reps 3 --stage demod prod generic \
  > $OUT/ab_c1536.jsonl 2> $OUT/ab_c1536.err || { tail $OUT/ab_c1536.err; exit 1; }
grep -v "^{" $OUT/ab_c1536.jsonl; grep '"rep": 2' $OUT/ab_c1536.jsonl | cut -c 1-260
timeout -k 10 300 python bench.py --C 1536 --frames 400 --no-cpu --no-mode-a --steps 10 --warmup 3 \
  > $OUT/bench_c1536.json 2> $OUT/bench_c1536.err || { tail $OUT/bench_c1536.err; exit 1; }
cut -c 1-400 $OUT/bench_c1536.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
