#!/bin/bash
# C=2048: part of the next row DMA'd into LDS (MRC2K_PF=1: 6+6 slabs,
# 2: 8+6, 3: 4+4) against the default kernel, same process; then the
# R=32 / prefix shapes through the same switch for parity.
set -o pipefail
mkdir -p gpurun_out/pf2k
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 64 --frames 400 --reps 5 --allocs 2 \
    default MRC2K_PF=1 MRC2K_PF=2 MRC2K_PF=3 > gpurun_out/pf2k/ab.txt 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 16 --frames 200 --reps 3 \
    default MRC2K_PF=1 MRC2K_PF=2 > gpurun_out/pf2k/ab_r16.txt 2>&1
