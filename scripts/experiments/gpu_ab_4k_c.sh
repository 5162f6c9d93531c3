#!/usr/bin/env bash
# C=4096 compute-only variants: with / without barriers (bit 0) / Hc (bit 1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/ab4kc_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 3 default MRC4K_DBG=64 MRC4K_DBG=65 \
  MRC4K_DBG=66 MRC4K_DBG=89 > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
cat $OUT/*.jsonl
