# round 6 (s): estimator waves at s_setprio 3: prio = parked row 0 + that, hprio = HEAD + that, pre = HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6s; mkdir -p $OUT
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod pre prio hprio > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -3 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod pre prio hprio > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -3 $OUT/ab_head.jsonl
