#!/usr/bin/env bash
# Round 3's evidence session on one MI355X: parity suite + smoke, then for each
# MRC shape a rocprofv3 kernel-trace/stats run plus one FETCH_SIZE and one
# WRITE_SIZE PMC pass (scripts/gpu_profile.sh, summarised into profiles/ by
# scripts/pmc_summary.py), the bench lines of the same code in the same
# session (default shape with cpu_baseline, configs[2] C=2048, C=4096,
# configs[1], antenna split), and the ZF bench with its own trace + PMC passes.
# usage: bash scripts/gpu_round3.sh <tag> [skip-tests]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r3}
OUT=gpurun_out/round_$TAG; mkdir -p $OUT
if [ "$2" != skip-tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
prof() { t=$1; shift; mode=$1; shift
  bash scripts/gpu_profile.sh $t "$@" || { echo "profile $t failed"; exit 1; }
  cd "$ROOT"; python scripts/pmc_summary.py gpurun_out/prof_$t $t $mode > /dev/null || exit 1; echo "profile $t ok"; }
prof $TAG ""
prof ${TAG}_c2048 notraffic --R 64 --C 2048 --frames 1000
prof ${TAG}_c4096 notraffic --R 32 --C 4096 --frames 400
prof ${TAG}_cfg1 notraffic --R 16 --frames 100
mkdir -p $OUT/profiles && cp profiles/${TAG}* profiles/pmc_traffic.json $OUT/profiles/
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; tail -c 700 $OUT/$name.json; echo; [ $rc -eq 0 ]; }
run bench && run bench_c2048 --no-cpu --steps 10 --R 64 --C 2048 --frames 1000 && \
run bench_c4096 --no-cpu --steps 10 --R 32 --C 4096 --frames 400 && \
run bench_cfg1 --no-cpu --no-mode-a --R 16 --frames 100 && \
run bench_split --no-cpu --mode split --steps 10 || exit 1
# zero forcing: bench, kernel trace, HBM counters at U = 16
ZOUT=$OUT/zf; mkdir -p $ZOUT
timeout -k 10 300 python -u scripts/zf_bench.py > $ZOUT/bench.json 2> $ZOUT/bench.err || { tail -5 $ZOUT/bench.err; exit 1; }
cat $ZOUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$ZOUT/trace" -o zf \
  -- python3 "$ROOT/scripts/zf_bench.py" --U 16 --no-cpu --reps 5 > "$ROOT/$ZOUT/trace.log" 2>&1 || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$ZOUT/pmc_$ctr" -o zf \
    -- python3 "$ROOT/scripts/zf_bench.py" --U 16 --no-cpu --reps 2 > "$ROOT/$ZOUT/pmc_$ctr.log" 2>&1 || exit 1
done
echo "round $TAG done"
