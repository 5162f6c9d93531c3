#!/bin/bash
# C=2048 receiver built with the ILP machine scheduler (Makefile KFLAGS):
# parity, same-box comparison with the default-scheduler build (lib "base"),
# then the configs[2] profile + bench line of the new build.
# SKIP_TESTS=1: only the LS comparison, bench and profile.
set -e -o pipefail
mkdir -p gpurun_out/ilp2k
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -k "2048" -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/ilp2k/gpu_2048.log 2>&1
  timeout -k 10 400 python -u scripts/libab.py --reps 3 --shapes 2048:64:400 prod base > gpurun_out/ilp2k/mrc.txt 2>&1
fi
timeout -k 10 300 python -u scripts/libab.py --reps 2 --shapes 2048:64:400 --extra=--ls prod base > gpurun_out/ilp2k/ls.txt 2>&1
timeout -k 10 300 python -u bench.py --C 2048 --R 64 --frames 1000 --no-cpu --no-mode-a > gpurun_out/ilp2k/bench.json 2> gpurun_out/ilp2k/bench.err
bash scripts/experiments/gpu_prof_cfg.sh r2f_c2048 --C 2048 --R 64 --frames 1000 > gpurun_out/ilp2k/prof.txt 2>&1
