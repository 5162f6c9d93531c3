#!/usr/bin/env bash
# C=2048 wave-pair MRC kernel: parity tests touching C=2048, then same-process
# A/B against the one-wave-per-symbol kernel (A/B build, MRC2K_PAIR=0).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/pair2k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "2048 and not 1000" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 64 --frames 200 --reps 3 default MRC2K_PAIR=0 > $OUT/ab_r64.jsonl 2>&1 || { cat $OUT/ab_r64.jsonl; exit 1; }
cat $OUT/ab_r64.jsonl
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 16 --frames 400 --reps 3 default MRC2K_PAIR=0 > $OUT/ab_r16.jsonl 2>&1 || { cat $OUT/ab_r16.jsonl; exit 1; }
cat $OUT/ab_r16.jsonl
