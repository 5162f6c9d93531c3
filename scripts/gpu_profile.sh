#!/usr/bin/env bash
# Profile bench.py on one MI355X: kernel-trace stats, then one PMC pass per
# counter (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md rocprofv3 section).
# usage: bash scripts/gpu_profile.sh <tag> [bench args...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}; shift || true
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu --no-mode-a "$@" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$ctr" -o run \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-mode-a "$@" > "$OUT/bench_$ctr.json" 2> "$OUT/bench_$ctr.err" || exit 1
done
echo "profile $TAG done"
