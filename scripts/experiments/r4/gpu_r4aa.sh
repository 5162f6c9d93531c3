# Round 4 session aa: C = 1536 receiver A/B -- product (next row prefetched
# in registers, 2 waves/SIMD) vs variant "np" (no register prefetch, 3 waves/SIMD).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4aa; mkdir -p $OUT
timeout -k 10 240 python scripts/abx.py --C 1536 --R 64 --frames 300 --reps 4 --stage demod prod np \
  > $OUT/ab_c1536.jsonl 2> $OUT/ab_c1536.err || { tail $OUT/ab_c1536.err; exit 1; }
grep -v "^{" $OUT/ab_c1536.jsonl; grep '"rep": 3' $OUT/ab_c1536.jsonl | cut -c 1-240
