#!/usr/bin/env bash
# Round-4 profile of ONE bench.py command (the credited driver form by
# default): the un-profiled run first (its bench line), then the SAME command
# under rocprofv3 --kernel-trace --stats (its own bench line comes from the
# profiled process, so the profiled kernel time is measured inside that run's
# ms_per_step), then one --pmc pass each for FETCH_SIZE, WRITE_SIZE and
# GRBM_GUI_ACTIVE + SQ counters (clock and wave-state fractions).
# usage: bash scripts/gpu_prof_r4.sh <tag> [bench args...]   (default: --gpus 1 --steps 20 --warmup 5)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r4}; shift || true
ARGS="$@"; [ -z "$ARGS" ] && ARGS="--gpus 1 --steps 20 --warmup 5"
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
echo "$ARGS" > "$OUT/args.txt"
timeout -k 10 300 python3 "$ROOT/scripts/clock_sampler.py" "$OUT/clock_unprofiled.jsonl" -- \
  python3 "$ROOT/bench.py" $ARGS > "$OUT/bench_unprofiled.json" 2> "$OUT/bench_unprofiled.err" || { tail "$OUT/bench_unprofiled.err"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$ROOT/bench.py" $ARGS --no-box > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || { tail "$OUT/bench_trace.err"; exit 1; }
PMC_ARGS="$ARGS --no-cpu --no-mode-a --no-box"
for ctr in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"; do
  name=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT/pmc_$name" -o run \
    -- python3 "$ROOT/bench.py" $PMC_ARGS > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { tail "$OUT/bench_$name.err"; exit 1; }
done
echo "profile $TAG done"
