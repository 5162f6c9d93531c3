#!/usr/bin/env bash
# A/B: the C=1024 row prefetch as 16 buffer loads with nt on every one
# (DEMOD_LOAD=1 / MRC1K_DBG=128) or none (2 / 256), against the product's
# __builtin_nontemporal_load form (the compiler keeps nt on 8-11 of 16).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3v2; mkdir -p $OUT
export OFDM_LSMRC_LIB=ab
for shape in "64 400" "16 100" "64 1250" "16 400"; do
  set -- $shape
  timeout -k 10 200 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 15 default DEMOD_LOAD=1 DEMOD_LOAD=2 >> $OUT/demod.jsonl 2> $OUT/demod_$1_$2.err || exit 1
done
timeout -k 10 200 python -u scripts/ab.py --R 64 --frames 400 --reps 15 default MRC1K_DBG=128 MRC1K_DBG=256 >> $OUT/mrc.jsonl 2> $OUT/mrc.err || exit 1
cat $OUT/demod.jsonl $OUT/mrc.jsonl | python -c "import sys,json; [print(d['variant'],d['R'],d['frames'],d['ms'],d['TBps'],d['qpsk_errors'],d['max_abs_diff_vs_first']) for d in map(json.loads,sys.stdin)]"
