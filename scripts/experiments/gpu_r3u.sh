#!/usr/bin/env bash
# A/B: one-launch bench timing with events at both ends of the loop (default)
# vs an event after every step (--step-events), default shape and configs[1].
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3u; mkdir -p $OUT
for rep in 1 2; do
  for mode in ends step; do
    ex=""; [ $mode = step ] && ex="--step-events"
    timeout -k 10 200 python -u bench.py --no-cpu --no-mode-a $ex > $OUT/def_${mode}_$rep.json 2> $OUT/def_${mode}_$rep.err || exit 1
    timeout -k 10 200 python -u bench.py --no-cpu --no-mode-a --R 16 --frames 100 --steps 50 $ex > $OUT/cfg1_${mode}_$rep.json 2> $OUT/cfg1_${mode}_$rep.err || exit 1
    echo "$rep $mode done"
  done
done
