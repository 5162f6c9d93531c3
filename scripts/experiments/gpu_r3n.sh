#!/usr/bin/env bash
# One-launch demod at C = 2048 / 4096 (k_demod_td2048 / 4096): its tests,
# the hand-off diagnostic, a same-process A/B against two launches, then
# the whole GPU suite.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3n}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_demod_onelaunch_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_onelaunch.log 2>&1 || { tail -40 $OUT/pytest_onelaunch.log; exit 1; }
tail -2 $OUT/pytest_onelaunch.log
for C in 2048 4096; do
  timeout -k 10 200 python -u scripts/demod_race.py $C 9 3 >> $OUT/race.log 2>&1 || { tail -20 $OUT/race.log; exit 1; }
done
tail -4 $OUT/race.log
timeout -k 10 300 python -u scripts/ab.py --demod --C 2048 --R 64 --frames 200 --reps 5 default DEMOD_FUSED=0 >> $OUT/ab_demod.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
timeout -k 10 300 python -u scripts/ab.py --demod --C 4096 --R 32 --frames 300 --reps 5 default DEMOD_FUSED=0 >> $OUT/ab_demod.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
cut -c1-200 $OUT/ab_demod.jsonl
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; exit $rc
