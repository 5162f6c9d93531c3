#!/usr/bin/env bash
# A/B: one-launch estimator with / without the next pilot row prefetched
# (OFDM_AB_DEMOD_LSPF), A/B build, same process; then the GPU one-launch tests
# on the A/B library's default variant is not needed (product tests follow).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3y; mkdir -p $OUT
export OFDM_LSMRC_LIB=ab
for shape in "16 100" "16 40" "16 200" "64 100" "64 400"; do
  set -- $shape
  timeout -k 10 200 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 15 default DEMOD_LSPF=0 >> $OUT/ab.jsonl 2> $OUT/ab_$1_$2.err || exit 1
done
cat $OUT/ab.jsonl | python -c "import sys,json; [print(d['variant'],d['R'],d['frames'],d['ms'],d['TBps'],d['qpsk_errors'],d['max_abs_diff_vs_first']) for d in map(json.loads,sys.stdin)]"
