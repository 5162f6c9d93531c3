#!/usr/bin/env bash
# Frequency-domain LS + MRC (SURVEY.md 8(d) mode A) in one GPU session:
# its parity tests, rocprofv3 stats + FETCH/WRITE PMC of bench.py --mode freq
# (summarised into profiles/<tag>_freq_*), then the un-profiled bench lines.
# usage: bash scripts/experiments/gpu_freq.sh <tag>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r2}
OUT=gpurun_out/freq_$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "freq" --timeout 120 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/gpu_profile.sh ${TAG}_freq --mode freq || { echo "profile failed"; exit 1; }
cd "$ROOT"; python scripts/pmc_summary.py gpurun_out/prof_${TAG}_freq ${TAG}_freq notraffic > /dev/null || exit 1
bash scripts/gpu_profile.sh ${TAG}_freq_c4096 --mode freq --R 32 --C 4096 --frames 400 || { echo "profile failed"; exit 1; }
cd "$ROOT"; python scripts/pmc_summary.py gpurun_out/prof_${TAG}_freq_c4096 ${TAG}_freq_c4096 notraffic > /dev/null || exit 1
mkdir -p $OUT/profiles && cp profiles/${TAG}_freq* $OUT/profiles/
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; tail -c 700 $OUT/$name.json; echo; [ $rc -eq 0 ]; }
run bench_freq --mode freq && run bench_freq_c2048 --mode freq --no-cpu --steps 10 --R 64 --C 2048 --frames 1000 && \
run bench_freq_c4096 --mode freq --no-cpu --steps 10 --R 32 --C 4096 --frames 400 && \
run bench_freq_r16 --mode freq --no-cpu --steps 20 --R 16 --C 1024 --frames 100
