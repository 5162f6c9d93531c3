# round 6 (m2): prod = lane recomputed per row + row 0 by LDS-DMA before the estimate wait; ln = lane only; pre = HEAD
# scratch per lane): one-launch tests, same-process A/B at configs[1] and the headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6m2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod ln pre > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -4 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod ln pre > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -4 $OUT/ab_head.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage combine prod ln pre > $OUT/ab_cfg1_comb.jsonl 2> $OUT/ab_cfg1_comb.err || { tail $OUT/ab_cfg1_comb.err; exit 1; }
tail -4 $OUT/ab_cfg1_comb.jsonl
