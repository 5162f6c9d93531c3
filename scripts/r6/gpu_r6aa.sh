# round 6 (aa): C = 4096 block start in one memory round trip (table loads before the ticket, row 0 / Hc row 0 /
# twiddle bases / tables in flight together) = prod vs pre (HEAD): tests, A/B at R = 32 x 400 (two orders) and
# the 50-frame partial launches
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6aa; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_demod_onelaunch_gpu.py tests/test_antenna_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c4k.jsonl 2> $OUT/ab_c4k.err || { tail $OUT/ab_c4k.err; exit 1; }
tail -2 $OUT/ab_c4k.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine pre prod > $OUT/ab_c4kb.jsonl 2> $OUT/ab_c4kb.err || { tail $OUT/ab_c4kb.err; exit 1; }
tail -2 $OUT/ab_c4kb.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 50 --reps 7 --launches 10 --stage partial prod pre > $OUT/ab_part.jsonl 2> $OUT/ab_part.err || { tail $OUT/ab_part.err; exit 1; }
tail -2 $OUT/ab_part.jsonl
