#!/usr/bin/env bash
# C=4096: the row loads alone (bit 7; +bit 0 without the per-row barrier)
# against the default and the compute-only variant (bit 6).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/ab4kmem_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 4 default MRC4K_DBG=128 MRC4K_DBG=129 \
  MRC4K_DBG=64 > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
cat $OUT/*.jsonl
