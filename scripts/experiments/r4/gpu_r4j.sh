# Round 4 session j: the fused any-C MRC (k_mrc_any) and the batched pilot FFT:
# any-C tests, the GPU suite, then the any-C throughput sweep (R = 64, 400
# frames) and a kernel-trace profile of the C = 1536 run.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${TAG:-r4j}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_any_c_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_any_c.log 2>&1 || { tail -60 $OUT/pytest_any_c.log; exit 1; }
tail -2 $OUT/pytest_any_c.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in 1536 600 1200 3000 3072 6144 8192 512 256; do
  timeout -k 10 300 python bench.py --C $C --frames 400 --no-cpu --no-mode-a --steps 10 --warmup 3 \
    > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || { tail $OUT/bench_c$C.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_c$C.json').read().strip().splitlines()[-1]); print($C, round(d['value']), round(d['ms_per_step'],3), d['check'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof1536 -o run -- python3 bench.py \
  --C 1536 --frames 400 --no-cpu --no-mode-a --steps 10 --warmup 3 > $OUT/prof1536.json 2> $OUT/prof1536.err \
  || { tail $OUT/prof1536.err; exit 1; }
find $OUT/prof1536 -name "*kernel_stats.csv" -exec cut -c 1-160 {} \;
