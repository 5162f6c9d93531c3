# Round 4 session w: the C = 512 receiver (one wave per symbol, frame_td1536.hip):
# any-C tests, same-process A/B at C = 512 against the generic any-C
# kernel (variant "generic" = the library before the 512 receiver, so its
# other sizes use their receivers too), bench lines, then the GPU suite.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4w; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_any_c_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_any_c.log 2>&1 || { tail -60 $OUT/pytest_any_c.log; exit 1; }
tail -2 $OUT/pytest_any_c.log
timeout -k 10 240 python scripts/abx.py --C 512 --R 64 --frames 400 --reps 3 --stage demod prod generic \
  > $OUT/ab_c512.jsonl 2> $OUT/ab_c512.err || { tail $OUT/ab_c512.err; exit 1; }
grep -v "^{" $OUT/ab_c512.jsonl; grep '"rep": 2' $OUT/ab_c512.jsonl | cut -c 1-260
for C in 512; do
  timeout -k 10 300 python bench.py --C $C --frames 400 --no-cpu --no-mode-a --steps 10 --warmup 3 \
    > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || { tail $OUT/bench_c$C.err; exit 1; }
  cut -c 1-200 $OUT/bench_c$C.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
