#!/usr/bin/env bash
# One-launch C=1024 demod (k_demod_td1024): its GPU tests, then a
# same-process A/B of frame_demod (LS + MRC) one launch vs two launches at
# configs[1] and the headline shape, then the whole GPU suite.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3h}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_demod_onelaunch_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_onelaunch.log 2>&1 || { tail -40 $OUT/pytest_onelaunch.log; exit 1; }
tail -3 $OUT/pytest_onelaunch.log
for shape in "16 100" "64 1250"; do
  set -- $shape
  timeout -k 10 300 python -u scripts/ab.py --demod --R $1 --frames $2 --reps 5 default DEMOD1K_FUSED=0 >> $OUT/ab_demod.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
done
cut -c1-230 $OUT/ab_demod.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; exit $rc
