# round 6 (at): reciprocal normalisation in the C = 2048 / 4096 / 512 / 1536 / 3072 / 6144 receivers (prod) vs
# pre (HEAD): GPU suite, A/B per size
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6at; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c4k.jsonl 2> $OUT/ab_c4k.err || { tail $OUT/ab_c4k.err; exit 1; }
tail -2 $OUT/ab_c4k.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine pre prod > $OUT/ab_c4kb.jsonl 2> $OUT/ab_c4kb.err || { tail $OUT/ab_c4kb.err; exit 1; }
tail -2 $OUT/ab_c4kb.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 2048 --R 64 --frames 400 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c2k.jsonl 2> $OUT/ab_c2k.err || { tail $OUT/ab_c2k.err; exit 1; }
tail -2 $OUT/ab_c2k.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 3072 --R 64 --frames 200 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c3k.jsonl 2> $OUT/ab_c3k.err || { tail $OUT/ab_c3k.err; exit 1; }
tail -2 $OUT/ab_c3k.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 512 --R 64 --frames 400 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c512.jsonl 2> $OUT/ab_c512.err || { tail $OUT/ab_c512.err; exit 1; }
tail -2 $OUT/ab_c512.jsonl
