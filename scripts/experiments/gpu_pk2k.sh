#!/bin/bash
# C=2048 receiver with packed row_fft_b + MAC (PK=6) as the default: C=2048 parity
# tests, then the configs[2] bench line and profile of the product build.
set -e -o pipefail
mkdir -p gpurun_out/pk2k
timeout -k 10 400 python -u -m pytest tests -m gpu -k "2048" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pk2k/gpu_2048.log 2>&1
timeout -k 10 300 python -u bench.py --C 2048 --R 64 --frames 1000 --no-cpu --no-mode-a > gpurun_out/pk2k/bench.json 2> gpurun_out/pk2k/bench.err
bash scripts/experiments/gpu_prof_cfg.sh r2h_c2048 --C 2048 --R 64 --frames 1000 > gpurun_out/pk2k/prof.txt 2>&1
