#!/usr/bin/env bash
# Product build (batched epilogue |H|^2 loads at C = 1024 / 2048) vs the
# round-3 HEAD build (lib/libofdm_lsmrc_r3head.so), one process per
# (shape, build), interleaved (scripts/libab.py).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3g}; mkdir -p $OUT
timeout -k 10 900 python -u scripts/libab.py --reps 3 --shapes 1024:16:100,1024:64:400,2048:64:200 prod r3head > $OUT/libab.jsonl 2> $OUT/libab.err || { tail -5 $OUT/libab.err; exit 1; }
cut -c1-200 $OUT/libab.jsonl
