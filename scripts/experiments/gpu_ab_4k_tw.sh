#!/usr/bin/env bash
# C=4096 twiddles by recurrence (MRC4K_PF bit 2 first FFT half, bit 3 second)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/ab4ktw_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 3 default MRC4K_PF=4 MRC4K_PF=8 \
  MRC4K_PF=12 MRC4K_PF=14 MRC4K_PF=76 > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
cat $OUT/*.jsonl
