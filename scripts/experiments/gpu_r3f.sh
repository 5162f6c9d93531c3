#!/usr/bin/env bash
# C=1024 receiver A/B: persistent grid (default) vs one block per workgroup
# (MRC1K_PERS=0), both with the batched |H|^2 epilogue loads, vs the
# round-3 HEAD build (lib/libofdm_lsmrc_r3head.so: serial epilogue loads);
# configs[1] and the headline shape.  Then the C=1024 GPU parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3f}; mkdir -p $OUT
for shape in "16 100" "64 400"; do
  set -- $shape
  for rep in 1 2; do
    timeout -k 10 200 python -u scripts/ab.py --R $1 --frames $2 --reps 3 default MRC1K_PERS=0 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    OFDM_LSMRC_LIB=r3head timeout -k 10 200 python -u scripts/ab.py --R $1 --frames $2 --reps 3 default >> $OUT/ab_head.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  done
done
cat $OUT/ab.jsonl $OUT/ab_head.jsonl | cut -c1-220
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; exit $rc
