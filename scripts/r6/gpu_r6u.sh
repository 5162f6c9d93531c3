# round 6 (u): B = the receivers' row loop takes its lane once per unit (lane-derived values hoisted: 745 instead
# of 768 instructions per row, 2 scratch accesses per row) vs prod (HEAD): A/B at configs[1], the headline, combine
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6u; mkdir -p $OUT
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod B > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -2 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod B > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -2 $OUT/ab_head.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 400 --reps 5 --launches 5 --stage combine prod B > $OUT/ab_comb.jsonl 2> $OUT/ab_comb.err || { tail $OUT/ab_comb.err; exit 1; }
tail -2 $OUT/ab_comb.jsonl
