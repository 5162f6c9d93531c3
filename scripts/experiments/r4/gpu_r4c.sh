# Round 4: GPU suite + smoke + default bench (driver form), then same-process
# library A/B (scripts/abx.py) of the packed-asm pad removal at C = 4096 / 2048.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r4c}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python scripts/abx.py --C 4096 --R 32 --frames 300 --reps 4 prod pk1 pk2 > $OUT/abx_c4096.jsonl 2>&1 || { tail $OUT/abx_c4096.jsonl; exit 1; }
tail -2 $OUT/abx_c4096.jsonl
timeout -k 10 300 python scripts/abx.py --C 2048 --R 64 --frames 200 --reps 4 prod pk1 pk2 > $OUT/abx_c2048.jsonl 2>&1 || { tail $OUT/abx_c2048.jsonl; exit 1; }
tail -2 $OUT/abx_c2048.jsonl
