#!/usr/bin/env bash
# Re-check: one-launch demod with row 0 DMA'd into LDS (MRC1K_R0=1) vs the
# product (row 0 by register load), A/B build, same process.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3z3; mkdir -p $OUT
export OFDM_LSMRC_LIB=ab
for shape in "16 100" "64 1250" "16 400"; do
  set -- $shape
  timeout -k 10 200 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 15 default MRC1K_R0=1 >> $OUT/ab.jsonl 2> $OUT/ab_$1_$2.err || exit 1
done
python -c "import sys,json; [print(d['variant'],d['R'],d['frames'],d['ms'],d['TBps'],d['max_abs_diff_vs_first']) for d in map(json.loads,open(sys.argv[1]))]" $OUT/ab.jsonl
