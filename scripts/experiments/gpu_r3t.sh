#!/usr/bin/env bash
# C=4096: one workgroup barrier per row (MRC4K_SW=1: the pair's images swap
# roles every row) vs two, same process, full receiver and partial
# numerators; outputs compared bit for bit (ab.py max_abs_diff_vs_first).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3t}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 7 default MRC4K_SW=1 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 400 --reps 5 default MRC4K_SW=1 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
timeout -k 10 300 python -u scripts/ab.py --partial --C 4096 --R 32 --frames 300 --reps 5 default MRC4K_SW=1 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['R'], d['frames'], d['variant'], d['ms'], d['frac_8TBps'], d['all_ms'], d['max_abs_diff_vs_first'], d['qpsk_errors'])"
