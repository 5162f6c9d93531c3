#!/usr/bin/env bash
# Diagnostic A/B of the three fused MRC kernels (A/B build, scripts/ab.py):
# default vs no barriers / no Hc / no stores, plus the read-bandwidth probe of
# the same box.  usage: bash scripts/experiments/gpu_ab_diag.sh <tag>
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/abdiag_${1:-x}; mkdir -p $OUT
timeout -k 10 120 ./scripts/bwprobe2 > $OUT/bwprobe2.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 1024 --R 64 --frames 400 default MRC1K_DBG=1 MRC1K_DBG=2 \
  MRC1K_DBG=4 MRC1K_DBG=6 > $OUT/c1024.jsonl 2> $OUT/c1024.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 64 --frames 300 default MRC2K_DBG=2 MRC2K_DBG=4 \
  MRC2K_DBG=6 > $OUT/c2048.jsonl 2> $OUT/c2048.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 default MRC4K_DBG=1 MRC4K_DBG=2 \
  MRC4K_DBG=4 MRC4K_DBG=6 > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
cat $OUT/bwprobe2.txt $OUT/*.jsonl
