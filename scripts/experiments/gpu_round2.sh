#!/usr/bin/env bash
# One GPU session for the round's evidence: parity suite, then for each MRC
# shape a rocprofv3 kernel-trace/stats run plus one FETCH_SIZE and one
# WRITE_SIZE PMC pass (scripts/gpu_profile.sh, summarised into profiles/ by
# scripts/pmc_summary.py), then the bench lines of the same code in the same
# session: the default shape (configs[3] slice, with cpu_baseline), configs[2]
# (R=64, C=2048, 1000 frames), R=32 x C=4096 (configs[4]'s per-GPU shape, full
# receiver) and the antenna-split mode.
# usage: bash scripts/gpu_round2.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r2}
OUT=gpurun_out/round_$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/gpu_profile.sh $TAG || { echo "profile $TAG failed"; exit 1; }
cd "$ROOT"; python scripts/pmc_summary.py gpurun_out/prof_$TAG $TAG > /dev/null || exit 1
bash scripts/gpu_profile.sh ${TAG}_c2048 --R 64 --C 2048 --frames 1000 || { echo "profile c2048 failed"; exit 1; }
cd "$ROOT"; python scripts/pmc_summary.py gpurun_out/prof_${TAG}_c2048 ${TAG}_c2048 notraffic > /dev/null || exit 1
bash scripts/gpu_profile.sh ${TAG}_c4096 --R 32 --C 4096 --frames 400 || { echo "profile c4096 failed"; exit 1; }
cd "$ROOT"; python scripts/pmc_summary.py gpurun_out/prof_${TAG}_c4096 ${TAG}_c4096 notraffic > /dev/null || exit 1
mkdir -p $OUT/profiles && cp profiles/${TAG}* profiles/pmc_traffic.json $OUT/profiles/
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; tail -c 600 $OUT/$name.json; echo; [ $rc -eq 0 ]; }
run bench && run bench_c2048 --no-cpu --steps 10 --R 64 --C 2048 --frames 1000 && \
run bench_c4096 --no-cpu --steps 10 --R 32 --C 4096 --frames 400 && run bench_split --no-cpu --mode split
