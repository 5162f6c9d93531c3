#!/usr/bin/env bash
# ZF detect (k_zf_wstat, per-XCD chunks): input prefetch depth 3 (default)
# vs 2 (ZF_LDS=13) vs 1 (ZF_LDS=14) vs 5 (ZF_LDS=11), U = 16 and 32, same process.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3z6b; mkdir -p $OUT
for U in 16 32; do
  timeout -k 10 200 python -u scripts/zf_ab.py --U $U --reps 10 default ZF_LDS=13 ZF_LDS=14 ZF_LDS=11 >> $OUT/ab.jsonl 2> $OUT/ab_$U.err || exit 1
done
cat $OUT/ab.jsonl
