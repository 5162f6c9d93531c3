#!/usr/bin/env bash
# Third diagnostic round: compute-only (no IQ loads after the first row,
# bit 6) and no-store (bit 2, every accumulator component kept live) variants
# of the three MRC kernels, same process as the default.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/abdiag3_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab.py --C 1024 --R 64 --frames 400 --reps 4 default MRC1K_DBG=4 MRC1K_DBG=64 \
  MRC1K_DBG=2 > $OUT/c1024.jsonl 2> $OUT/c1024.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 64 --frames 200 --reps 4 default MRC2K_DBG=4 MRC2K_DBG=64 \
  MRC2K_DBG=2 > $OUT/c2048.jsonl 2> $OUT/c2048.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 4 default MRC4K_DBG=4 MRC4K_DBG=64 \
  MRC4K_DBG=1 MRC4K_DBG=2 > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
cat $OUT/*.jsonl
