# round 6 (n): split estimator without spills (two estimator workgroups per frame, the second to arrive adds the
# two |H|^2 parts; prod) vs HEAD (pre): GPU suite, same-process A/B at configs[1] and the headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6n; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod pre > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -3 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod pre > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -3 $OUT/ab_head.jsonl
