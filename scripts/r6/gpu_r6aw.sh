# round 6 (aw): LS divide by one reciprocal (ls_conj) = prod vs pre (HEAD): GPU suite, A/B configs[1] (two orders), headline, combine

set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6aw; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod pre > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -2 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod pre prod > $OUT/ab_cfg1b.jsonl 2> $OUT/ab_cfg1b.err || { tail $OUT/ab_cfg1b.err; exit 1; }
tail -2 $OUT/ab_cfg1b.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod pre > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -2 $OUT/ab_head.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage combine prod pre > $OUT/ab_comb.jsonl 2> $OUT/ab_comb.err || { tail $OUT/ab_comb.err; exit 1; }
tail -2 $OUT/ab_comb.jsonl
