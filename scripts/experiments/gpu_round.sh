#!/usr/bin/env bash
# One GPU session: parity tests, rocprofv3 profile (kernel trace + PMC passes),
# profiles/ summary, then the default bench line (with cpu_baseline).
# usage: bash scripts/gpu_round.sh <tag>      (outputs under gpurun_out/)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
bash scripts/gpu_profile.sh $TAG || { echo "profile failed"; exit 1; }
cd "$ROOT"
python scripts/pmc_summary.py gpurun_out/prof_$TAG $TAG > /dev/null || exit 1
mkdir -p gpurun_out/profiles_$TAG && cp profiles/${TAG}_* profiles/pmc_traffic.json gpurun_out/profiles_$TAG/
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; exit $rc
