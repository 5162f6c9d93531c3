# Round 4 session p: same-process A/B of the any-C row-group size (product:
# G = 1 row per group for 1024 < C <= 2048 and 2048 < C <= 4096; capg2: the
# next larger LDS variant, G = 2) on the receiver (estimate + fused MRC).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4p; mkdir -p $OUT
for C in 1536 3072 1200 3000 2048 6144; do
  timeout -k 10 240 python scripts/abx.py --C $C --R 64 --frames 200 --reps 3 --stage demod prod capg2 \
    > $OUT/ab_c$C.jsonl 2> $OUT/ab_c$C.err || { tail $OUT/ab_c$C.err; exit 1; }
  grep -v "^{" $OUT/ab_c$C.jsonl | cut -c 1-200
done
