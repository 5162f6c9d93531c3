#!/usr/bin/env bash
# After the ZF apply XCD-map default: GPU suite, then the ZF bench with its
# kernel trace and HBM counters at U = 16 (as in scripts/gpu_round3.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/${1:-r3m}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ZOUT=$OUT/zf; mkdir -p $ZOUT
timeout -k 10 300 python -u scripts/zf_bench.py > $ZOUT/bench.json 2> $ZOUT/bench.err || { tail -5 $ZOUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$ZOUT/trace" -o zf \
  -- python3 "$ROOT/scripts/zf_bench.py" --U 16 --no-cpu --reps 5 > "$ROOT/$ZOUT/trace.log" 2>&1 || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$ZOUT/pmc_$ctr" -o zf \
    -- python3 "$ROOT/scripts/zf_bench.py" --U 16 --no-cpu --reps 2 > "$ROOT/$ZOUT/pmc_$ctr.log" 2>&1 || exit 1
done
echo "r3m done"
