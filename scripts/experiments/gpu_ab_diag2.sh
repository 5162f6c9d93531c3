#!/usr/bin/env bash
# Second diagnostic round: the C=1024 epilogue split (no stores / no |H|^2
# divides / nontemporal stores) and the C=4096 barriers one at a time.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/abdiag_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab.py --C 1024 --R 64 --frames 400 --reps 4 default MRC1K_DBG=4 MRC1K_DBG=8 \
  MRC1K_DBG=16 MRC1K_DBG=32 > $OUT/c1024.jsonl 2> $OUT/c1024.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 4 default MRC4K_DBG=1 MRC4K_DBG=8 \
  MRC4K_DBG=16 > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
cat $OUT/*.jsonl
