#!/usr/bin/env bash
# ZF apply (k_zf_apply_ws16) XCD maps, same process: default (chunk x
# subcarrier-block groups round-robin over XCDs, row blocks adjacent) vs
# every block of a symbol chunk on one XCD (ZF_A16=10: row blocks adjacent,
# 11: subcarrier blocks adjacent, 12: = 10 with 128-symbol chunks).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3k}; mkdir -p $OUT
for U in 16 8; do
  timeout -k 10 300 python -u scripts/zf_ab.py --U $U --reps 10 default ZF_A16=10 ZF_A16=11 ZF_A16=12 >> $OUT/zf_ab.jsonl 2>> $OUT/zf_ab.err || { tail -5 $OUT/zf_ab.err; exit 1; }
done
cat $OUT/zf_ab.jsonl | cut -c1-250
