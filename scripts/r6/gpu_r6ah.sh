# round 6 (ah): static rounds of the one-launch demod: st15 / st2 / st3 = 1.5 / 2 / 3 rounds static (half units
# for the last k0 blocks of each range after them), st2h = 2 static rounds with half units for k0/2; prod = HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6ah; mkdir -p $OUT
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod st15 st2 st2h st3 > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -5 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 300 --reps 7 --launches 10 --stage demod prod st15 st2 st2h st3 > $OUT/ab_r16f300.jsonl 2> $OUT/ab_r16f300.err || { tail $OUT/ab_r16f300.err; exit 1; }
tail -5 $OUT/ab_r16f300.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 100 --reps 7 --launches 10 --stage demod prod st15 st2 st2h st3 > $OUT/ab_r64f100.jsonl 2> $OUT/ab_r64f100.err || { tail $OUT/ab_r64f100.err; exit 1; }
tail -5 $OUT/ab_r64f100.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod st2 st3 > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -3 $OUT/ab_head.jsonl
