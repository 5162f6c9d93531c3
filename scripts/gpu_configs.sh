#!/usr/bin/env bash
# GPU tests + bench lines at the other BASELINE shapes (no CPU baseline).
# usage: bash scripts/gpu_configs.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-c1}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() { name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 10 "$@" > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err
  rc=$?; echo "$name rc=$rc"; cat gpurun_out/bench_${TAG}_$name.json; [ $rc -eq 0 ]; }
run cfg2 --frames 100 --R 16 && run cfg3 --frames 1000 --R 64 --C 2048 && run cfg5slice --frames 100 --R 32 --C 4096
