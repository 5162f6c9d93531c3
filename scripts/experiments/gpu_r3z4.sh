#!/usr/bin/env bash
# One-launch demod with row 0 by LDS-DMA after the fallback's address
# laundering (25 -> 6 spilled VGPRs) vs the product; plus the R0 fallback
# (bounded wait expired) against the default output.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3z4; mkdir -p $OUT
export OFDM_LSMRC_LIB=ab
for shape in "16 100" "64 1250" "16 400" "64 100"; do
  set -- $shape
  timeout -k 10 200 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 15 default MRC1K_R0=1 >> $OUT/ab.jsonl 2> $OUT/ab_$1_$2.err || exit 1
done
timeout -k 10 200 python -u scripts/ab.py --demod --R 16 --frames 20 --reps 2 default MRC1K_R0=1,DEMOD_SPIN=0 DEMOD_SPIN=0 >> $OUT/fallback.jsonl 2> $OUT/fallback.err || exit 1
python -c "import sys,json; [print(d['variant'],d['R'],d['frames'],d['ms'],d['TBps'],d['qpsk_errors'],d['max_abs_diff_vs_first']) for f in sys.argv[1:] for d in map(json.loads,open(f))]" $OUT/ab.jsonl $OUT/fallback.jsonl
