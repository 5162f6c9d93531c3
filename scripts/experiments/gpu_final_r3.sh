#!/usr/bin/env bash
# Round 3's closing evidence on one MI355X: GPU suite + smoke, rocprof +
# PMC of the default bench (one-launch C=1024) and configs[1], then the
# bench lines of every BASELINE shape from the same code in the same
# session (default with cpu_baseline, configs[1], configs[2] C=2048, the
# configs[4] slice C=4096, its antenna split).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; TAG=${1:-r3z}; OUT=gpurun_out/round_$TAG; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
prof() { t=$1; shift; mode=$1; shift
  bash scripts/gpu_profile.sh $t "$@" || { echo "profile $t failed"; exit 1; }
  cd "$ROOT"; python scripts/pmc_summary.py gpurun_out/prof_$t $t $mode > /dev/null || exit 1; echo "profile $t ok"; }
prof $TAG ""
prof ${TAG}_cfg1 notraffic --R 16 --frames 100
mkdir -p $OUT/profiles && cp profiles/${TAG}* profiles/pmc_traffic.json $OUT/profiles/
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; tail -c 400 $OUT/$name.json; echo; [ $rc -eq 0 ]; }
run bench && run bench_cfg1 --no-cpu --no-mode-a --R 16 --frames 100 --steps 200 --warmup 20 && \
run bench_c2048 --no-cpu --no-mode-a --steps 10 --R 64 --C 2048 --frames 1000 && \
run bench_c4096 --no-cpu --no-mode-a --steps 10 --R 32 --C 4096 --frames 400 && \
run bench_split --no-cpu --mode split --steps 10 || exit 1
echo "round $TAG done"
