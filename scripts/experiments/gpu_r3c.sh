#!/usr/bin/env bash
# configs[1] LS diagnostics: rocprof kernel trace of scripts/ab.py --ls with
# the LS1K_* A/B variants (R=16, 100 frames), then kernel durations per variant.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3c}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/ls_trace" -o run \
  -- python3 "$ROOT/scripts/ab.py" --ls --R 16 --frames 100 --reps 3 default LS1K_NW=4 LS1K_NW=8 LS1K_DBG=1 LS1K_DBG=2 LS1K_DBG=4 LS1K_DBG=6 \
  > "$ROOT/$OUT/ls_ab.jsonl" 2> "$ROOT/$OUT/ls_ab.err" || { tail -5 "$ROOT/$OUT/ls_ab.err"; exit 1; }
cat "$ROOT/$OUT/ls_ab.jsonl"
