#!/usr/bin/env bash
# pk.hpp single-statement complex ops vs the two-statement forms (OFDM_PK_SPLIT):
# the same A/B script in separate processes on one box, alternating builds.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/pkmerge; mkdir -p $OUT
L=gpu-accel-ofdm-ls-mrc_amd/lib
cp $L/libofdm_lsmrc_ab.so $OUT/merged.so
for i in 1 2; do
  for v in split merged; do
    if [ $v = split ]; then cp $L/libofdm_lsmrc_ab_split.so $L/libofdm_lsmrc_ab.so; else cp $OUT/merged.so $L/libofdm_lsmrc_ab.so; fi
    timeout -k 10 200 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 3 default 2>/dev/null | sed "s/\"variant\": \"default\"/\"variant\": \"$v\"/" >> $OUT/c4096.jsonl || exit 1
  done
done
cp $OUT/merged.so $L/libofdm_lsmrc_ab.so
cut -c1-140 $OUT/c4096.jsonl
