#!/usr/bin/env bash
# Build A/B: every row load plain (-DOFDM_ROW_NT=0, lib/libofdm_lsmrc_plain.so)
# vs the product's nontemporal row loads, alternating processes on one box.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3w2; mkdir -p $OUT
timeout -k 10 500 python -u scripts/libab.py --reps 3 prod plain > $OUT/mrc.jsonl 2> $OUT/mrc.err || exit 1
timeout -k 10 300 python -u scripts/libab.py --reps 3 --shapes 1024:64:1250,1024:16:100 --extra=--demod prod plain > $OUT/demod.jsonl 2> $OUT/demod.err || exit 1
grep -h "^{" $OUT/mrc.jsonl $OUT/demod.jsonl | python -c "import sys,json; [print(d['lib'],d['rep'],d['C'],d['R'],d['frames'],d['ms'],d['TBps']) for d in map(json.loads,sys.stdin)]"
