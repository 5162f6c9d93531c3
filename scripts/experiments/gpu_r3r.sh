#!/usr/bin/env bash
# GPU suite on the row-0-DMA product, then frame_demod one launch vs two
# launches (DEMOD_FUSED=0; its MRC now with the row-0 DMA), same process.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3r}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for shape in "16 100" "16 400" "64 100" "64 1250"; do
  set -- $shape
  timeout -k 10 300 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 7 default DEMOD_FUSED=0 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['R'], d['frames'], d['variant'], d['ms'], d['all_ms'], d['max_abs_diff_vs_first'])"
