#!/usr/bin/env bash
# C=4096: two independent 2-pair workgroups per CU with one Hc buffer
# (MRC4K_HP=2) vs one 4-pair workgroup with the double buffer (default).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/ab4khp_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 4 default MRC4K_HP=2 \
  > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 1 --partial default MRC4K_HP=2 \
  > $OUT/c4096p.jsonl 2> $OUT/c4096p.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 5 --S 8 --frames 40 --reps 1 default MRC4K_HP=2 \
  > $OUT/c4096s.jsonl 2> $OUT/c4096s.err || exit 1
cat $OUT/*.jsonl
