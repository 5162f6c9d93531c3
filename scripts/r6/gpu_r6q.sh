# round 6 (q): prod = receivers transform row 0 while the estimate is on its way (wait inside row 0; fallback
# estimate inside the wait: 376-404 B of scratch), split estimator; sx = HEAD + an unused 416-B private segment
# (is the scratch size itself a cost?); pre = HEAD.  One-launch tests, A/B at configs[1] and the headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6q; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod sx pre > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -4 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod sx pre > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -4 $OUT/ab_head.jsonl
