#!/usr/bin/env bash
# One-launch C=1024 flow evidence: rocprof + PMC of bench.py (default shape
# and configs[1], one launch per step), the bench lines of the same code
# (one-launch default and --flow two), and the whole GPU suite + smoke.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; TAG=${1:-r3j}; OUT=gpurun_out/round_$TAG; mkdir -p $OUT
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
  rc=$?; echo "$name rc=$rc"; tail -c 600 $OUT/$name.json; echo; [ $rc -eq 0 ]; }
run bench && run bench_two --no-cpu --no-mode-a --flow two && \
run bench_cfg1 --no-cpu --no-mode-a --R 16 --frames 100 --steps 50 && \
run bench_cfg1_two --no-cpu --no-mode-a --R 16 --frames 100 --steps 50 --flow two || exit 1
echo "round $TAG done"
