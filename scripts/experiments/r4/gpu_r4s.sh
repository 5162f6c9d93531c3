# Round 4 session s: same-process A/B of the per-wave fused any-C MRC
# (variant "wave": one wave per data symbol, stages in place with wave-level
# ordering, no workgroup barrier) against the product's workgroup kernel.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4s; mkdir -p $OUT
for C in 1536 1200 600 512 1000; do
  timeout -k 10 240 python scripts/abx.py --C $C --R 64 --frames 200 --reps 3 --stage demod prod wave \
    > $OUT/ab_c$C.jsonl 2> $OUT/ab_c$C.err || { tail $OUT/ab_c$C.err; exit 1; }
  grep -v "^{" $OUT/ab_c$C.jsonl | cut -c 1-200
  grep '"rep": 2' $OUT/ab_c$C.jsonl | cut -c 1-300
done
