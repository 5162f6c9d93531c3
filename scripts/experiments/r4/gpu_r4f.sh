# Round 4: row-group estimate flags of the one-launch C = 1024 demod: its GPU
# tests, then same-process A/B against the previous commit (base) at configs[1]
# and the headline shape; the bench line of configs[1] in the driver's form.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_gpu_parity.py tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python scripts/abx.py --stage demod --C 1024 --R 16 --frames 100 --reps 6 --launches 20 prod base > $OUT/abx_cfg1.jsonl 2>&1 || { tail $OUT/abx_cfg1.jsonl; exit 1; }
tail -2 $OUT/abx_cfg1.jsonl
timeout -k 10 300 python scripts/abx.py --stage demod --C 1024 --R 64 --frames 1250 --reps 4 prod base > $OUT/abx_r64.jsonl 2>&1 || { tail $OUT/abx_r64.jsonl; exit 1; }
tail -2 $OUT/abx_r64.jsonl
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --R 16 --frames 100 --no-cpu > $OUT/bench_cfg1.json 2>&1 || { tail $OUT/bench_cfg1.json; exit 1; }
tail -1 $OUT/bench_cfg1.json | cut -c 1-400
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-mode-a > $OUT/bench.json 2>&1 || { tail $OUT/bench.json; exit 1; }
tail -1 $OUT/bench.json | cut -c 1-400
