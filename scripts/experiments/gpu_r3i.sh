#!/usr/bin/env bash
# One-launch C=1024 demod: write-through publish (default) vs plain stores +
# release fence (DEMOD1K_WT=0) vs two launches (DEMOD1K_FUSED=0), same
# process, configs[1] and a mid-size batch; then its GPU tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3i}; mkdir -p $OUT
for shape in "16 100" "16 400" "64 100"; do
  set -- $shape
  timeout -k 10 300 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 7 default DEMOD1K_WT=0 DEMOD1K_FUSED=0 >> $OUT/ab_demod.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
done
cut -c1-150 $OUT/ab_demod.jsonl
timeout -k 10 300 python -u -m pytest tests/test_demod_onelaunch_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_onelaunch.log 2>&1; rc=$?
tail -3 $OUT/pytest_onelaunch.log; exit $rc
