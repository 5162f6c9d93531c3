#!/usr/bin/env bash
# Round 3 probes: ZF store-stream probe, rocprof kernel trace of the configs[1] bench.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3b}; mkdir -p $OUT
timeout -k 10 120 scripts/zfprobe2 > $OUT/zfprobe2.txt 2>&1 || { cat $OUT/zfprobe2.txt; exit 1; }
cat $OUT/zfprobe2.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/cfg1_trace" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-mode-a --R 16 --frames 100 \
  > "$ROOT/$OUT/cfg1_trace.json" 2> "$ROOT/$OUT/cfg1_trace.err" || exit 1
echo "trace done"
