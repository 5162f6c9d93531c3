#!/usr/bin/env bash
# GPU parity suite, then optional same-process A/B: scripts/gpu_check.sh <tag> [C R frames variants...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=gpurun_out/check_$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
if [ $# -ge 3 ]; then
  C=$1; R=$2; F=$3; shift 3
  timeout -k 10 300 python -u scripts/ab.py --C $C --R $R --frames $F --reps 3 "$@" > $OUT/ab.jsonl 2> $OUT/ab.err || exit 1
  cat $OUT/ab.jsonl
fi
