#!/usr/bin/env bash
# ZF apply XCD maps over U (same process): 8-row tiles (U <= 20) chunk groups
# round-robin (15 = today's default) vs a chunk's blocks on one XCD (10);
# 4-row tiles (U <= 40) likewise (14 vs 13).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3l}; mkdir -p $OUT
for U in 4 8 16 20; do
  timeout -k 10 300 python -u scripts/zf_ab.py --U $U --reps 10 ZF_A16=15 ZF_A16=10 ZF_A16=15 ZF_A16=10 >> $OUT/zf_ab.jsonl 2>> $OUT/zf_ab.err || { tail -5 $OUT/zf_ab.err; exit 1; }
done
for U in 24 32; do
  timeout -k 10 300 python -u scripts/zf_ab.py --U $U --reps 10 ZF_A16=14 ZF_A16=13 ZF_A16=14 ZF_A16=13 >> $OUT/zf_ab.jsonl 2>> $OUT/zf_ab.err || { tail -5 $OUT/zf_ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/zf_ab.jsonl'):
    d=json.loads(l); print(d['U'], d['variant'], d['apply_ms'], d['apply_frac'], d['max_rel_diff_vs_first'])"
