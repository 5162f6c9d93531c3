#!/usr/bin/env bash
# C=4096 wave-quad receiver (frame_td4096r.hip): parity tests at C=4096, then
# same-process A/B against the wave-pair kernel (A/B build, MRC4K_R=0).
# Stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/quad4k; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "4096" > $OUT/pytest.log 2>&1 \
  || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 3 --ls-per-variant MRC4K_R=1 MRC4K_R=68 default MRC4K_DBG=64 > $OUT/ab.jsonl 2>&1 \
  || { tail -20 $OUT/ab.jsonl; exit 1; }
cut -c1-250 $OUT/ab.jsonl
