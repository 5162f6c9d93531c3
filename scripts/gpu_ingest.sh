#!/usr/bin/env bash
# Streaming-ingest session: pipeline + ring tests, the whole GPU suite, the
# PCIe-inclusive bench and the ring ingest rate.  usage: bash scripts/gpu_ingest.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
TAG=${1:-ingest}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_pipeline_gpu.py tests/test_e2e_gpu.py > $OUT/pytest_new.log 2>&1
rc=$?; tail -30 $OUT/pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  > $OUT/pytest_all.log 2>&1
rc=$?; tail -3 $OUT/pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode pcie --steps 3 --warmup 1 > $OUT/bench_pcie.json 2> $OUT/bench_pcie.err
rc=$?; cat $OUT/bench_pcie.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/ring_bench.sh 100 > $OUT/ring.log 2>&1
rc=$?; cat $OUT/ring.log; exit $rc
