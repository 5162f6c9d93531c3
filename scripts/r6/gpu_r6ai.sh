# round 6 (ai): two static rounds for the C = 2048 / 4096 receivers too (s2k) vs prod: tests on s2k, A/B at
# C = 4096 R = 32 x 400 and x 50 (split mode's partial launches), C = 2048 R = 64 x 400 and R = 16 x 100
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6ai; mkdir -p $OUT
OFDM_LSMRC_LIB=s2k timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine prod s2k > $OUT/ab_c4k.jsonl 2> $OUT/ab_c4k.err || { tail $OUT/ab_c4k.err; exit 1; }
tail -2 $OUT/ab_c4k.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 50 --reps 7 --launches 10 --stage partial prod s2k > $OUT/ab_c4k_part.jsonl 2> $OUT/ab_c4k_part.err || { tail $OUT/ab_c4k_part.err; exit 1; }
tail -2 $OUT/ab_c4k_part.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 2048 --R 64 --frames 400 --reps 5 --launches 5 --stage combine prod s2k > $OUT/ab_c2k.jsonl 2> $OUT/ab_c2k.err || { tail $OUT/ab_c2k.err; exit 1; }
tail -2 $OUT/ab_c2k.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 2048 --R 16 --frames 100 --reps 9 --launches 10 --stage combine prod s2k > $OUT/ab_c2k_r16.jsonl 2> $OUT/ab_c2k_r16.err || { tail $OUT/ab_c2k_r16.err; exit 1; }
tail -2 $OUT/ab_c2k_r16.jsonl
