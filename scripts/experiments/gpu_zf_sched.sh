#!/bin/bash
# ZF apply/detect under three builds of the same sources (product, max-ilp,
# max-memory-clause machine scheduler), alternating processes on one box.
set -e -o pipefail
mkdir -p gpurun_out/zfsched
for rep in 1 2; do
  for lib in "" zilp zmc; do
    OFDM_LSMRC_LIB="$lib" timeout -k 10 200 python -u scripts/zf_bench.py --no-cpu --U 16 32 --reps 10 \
        > gpurun_out/zfsched/zf_${lib:-prod}_$rep.json 2> gpurun_out/zfsched/zf_${lib:-prod}_$rep.err
  done
done
