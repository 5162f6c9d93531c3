#!/bin/bash
# Final-tree GPU suite + smoke (product library), then the C=2048 A/B of the
# MRC kernel held to 3 waves/SIMD (MRC2K_W3=1) against the default (2).
set -o pipefail
mkdir -p gpurun_out/w3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/w3/gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/w3/smoke.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 64 --frames 400 --reps 5 --allocs 2 \
    default MRC2K_W3=1 MRC2K_DBG=64 MRC2K_W3=64 > gpurun_out/w3/ab_w3.txt 2>&1
