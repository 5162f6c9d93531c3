# Round 4 final check on the final library (after the receivers' non-temporal
# loads and per-symbol row pointers): full GPU suite, smoke, the driver's
# default bench line and bench lines at C = 1536 / 3072.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4aj; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
cut -c 1-200 $OUT/bench_default.json
for cfg in "1536 400" "3072 200"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --R 64 --C $1 --frames $2 \
    > $OUT/bench_c$1.json 2> $OUT/bench_c$1.err || { tail $OUT/bench_c$1.err; exit 1; }
  cut -c 1-200 $OUT/bench_c$1.json
done
