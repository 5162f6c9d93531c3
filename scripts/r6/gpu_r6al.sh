# round 6 (al): df = row-0 DMA and the flag look issued before the table store (with the table loads in flight)
# vs prod: one-launch tests on df, A/B at configs[1] (two orders), headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6al; mkdir -p $OUT
OFDM_LSMRC_LIB=df timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod df > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -2 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod df prod > $OUT/ab_cfg1b.jsonl 2> $OUT/ab_cfg1b.err || { tail $OUT/ab_cfg1b.err; exit 1; }
tail -2 $OUT/ab_cfg1b.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod df > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -2 $OUT/ab_head.jsonl
