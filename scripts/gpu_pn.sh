#!/usr/bin/env bash
# PN frame-sync session: its GPU tests, the correlator bench and a rocprofv3
# kernel-trace of it.  usage: bash scripts/gpu_pn.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
TAG=${1:-pn}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_pn_sync_gpu.py > $OUT/pytest_pn.log 2>&1
rc=$?; tail -20 $OUT/pytest_pn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/pn_bench.py > $OUT/pn_bench.json 2> $OUT/pn_bench.err
rc=$?; cat $OUT/pn_bench.json; [ $rc -eq 0 ] || { tail $OUT/pn_bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run \
  -- python3 "$ROOT/scripts/pn_bench.py" --reps 5 > "$ROOT/$OUT/prof_bench.json" 2> "$ROOT/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; exit $rc
