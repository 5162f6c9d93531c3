# round 6 (c): C = 4096 receiver with 16-B LDS accesses (prod) vs the same tree before it (pc):
# GPU suite, same-process A/B (R=32 x 400 combine, 50-frame partial), driver-form bench lines (frames, split)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 6 --launches 5 --stage combine prod pc > $OUT/ab_c4k.jsonl 2> $OUT/ab_c4k.err || { tail $OUT/ab_c4k.err; exit 1; }
tail -2 $OUT/ab_c4k.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 4096 --R 32 --frames 50 --reps 6 --launches 10 --stage partial prod pc > $OUT/ab_c4k_p50.jsonl 2> $OUT/ab_c4k_p50.err || { tail $OUT/ab_c4k_p50.err; exit 1; }
tail -2 $OUT/ab_c4k_p50.jsonl
timeout -k 10 300 python -u bench.py --C 4096 --R 32 --frames 400 --steps 20 --warmup 5 --no-cpu > $OUT/bench_c4096.json 2> $OUT/bench_c4096.err || { tail $OUT/bench_c4096.err; exit 1; }
tail -c 600 $OUT/bench_c4096.json
timeout -k 10 300 python -u bench.py --mode split --steps 20 --warmup 5 --no-cpu > $OUT/bench_split.json 2> $OUT/bench_split.err || { tail $OUT/bench_split.err; exit 1; }
tail -c 400 $OUT/bench_split.json
