#!/usr/bin/env bash
# Bench lines of the final code at every BASELINE shape (no CPU baseline,
# no GPU suite): configs[1] R=16 10k symbols, configs[2] C=2048 R=64 100k,
# configs[3] default (N=1 slice), configs[4] antenna split (N=1 slice), PCIe.
# usage: bash scripts/gpu_configs_final.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/cfg_${1:-final}; mkdir -p $OUT
run() { name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 "$@" > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; cat $OUT/$name.json; [ $rc -eq 0 ]; }
run cfg1_r16 --frames 100 --R 16 && run cfg2_c2048 --frames 1000 --R 64 --C 2048 && \
run cfg4_split --mode split && run pcie --mode pcie
