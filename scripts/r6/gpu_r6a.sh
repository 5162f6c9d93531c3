# round 6 (a): tagged work-ticket counters -- GPU suite, then same-process A/B vs the round-5 build (r5)
# prod = tagged tickets + split estimator (nh = 2 at configs[1]); tk = tagged tickets only (commit 9a79e08); r5 = round-5 final
# at configs[1] (C=1024 R=16 x 100, one-launch demod), the headline (R=64 x 1250) and C=4096 R=32 x 400
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 9 --launches 20 --stage demod prod tk r5 > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -3 $OUT/ab_cfg1.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod tk r5 > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -3 $OUT/ab_head.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine prod r5 > $OUT/ab_c4k.jsonl 2> $OUT/ab_c4k.err || { tail $OUT/ab_c4k.err; exit 1; }
tail -2 $OUT/ab_c4k.jsonl
