#!/usr/bin/env bash
# Round 3 GPU session: parity suite + smoke, then bench lines.
# usage: [AB="ab.py args"] bash scripts/experiments/gpu_r3.sh <tag> [bench-set]
#   bench-set: "base" (default: headline + split + configs[1] + C=4096) or "none"
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r3}; SET=${2:-base}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
[ "$SET" = none ] && exit 0
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; echo "$name rc=$rc"; tail -c 400 $OUT/$name.json; echo; [ $rc -eq 0 ]; }
run bench && run bench_split --no-cpu --mode split --steps 10 && \
run bench_cfg1 --no-cpu --no-mode-a --R 16 --frames 100 && \
run bench_c4096 --no-cpu --steps 10 --R 32 --C 4096 --frames 400
[ $? -eq 0 ] || exit 1
timeout -k 10 300 bash scripts/ring_bench.sh 20 > $OUT/ring.log 2>&1; rc=$?; tail -5 $OUT/ring.log; [ $rc -eq 0 ] || exit $rc
if [ -x scripts/wrprobe ]; then timeout -k 10 120 scripts/wrprobe > $OUT/wrprobe.txt 2>&1 || exit 1; cat $OUT/wrprobe.txt; fi
if [ -n "$AB" ]; then
  timeout -k 10 400 python -u scripts/ab.py $AB > $OUT/ab.jsonl 2> $OUT/ab.err; rc=$?; cat $OUT/ab.jsonl; exit $rc
fi
