#!/usr/bin/env bash
# C=1024 row 0 by LDS-DMA (MRC1K_R0=1) vs register load, same process:
# the two-launch MRC (frame_combine) and the one-launch demod, configs[1]
# and the headline shape.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3p}; mkdir -p $OUT
for shape in "16 100" "64 400"; do
  set -- $shape
  timeout -k 10 300 python -u scripts/ab.py --R $1 --frames $2 --reps 7 default MRC1K_R0=1 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  timeout -k 10 300 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 7 default MRC1K_R0=1 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['R'], d['frames'], d['variant'], d['ms'], d['all_ms'], d['max_abs_diff_vs_first'], d['qpsk_errors'])"
