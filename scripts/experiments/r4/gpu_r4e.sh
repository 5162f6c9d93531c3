# Round 4 evidence session: GPU suite on the current product library, then the
# driver-form profile of the default bench and profiles of the C = 4096 slice,
# configs[1] and the antenna split.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash scripts/gpu_prof_r4.sh r4e || exit 1
bash scripts/gpu_prof_r4.sh r4e_c4096 --gpus 1 --steps 20 --warmup 5 --R 32 --C 4096 --frames 400 || exit 1
bash scripts/gpu_prof_r4.sh r4e_cfg1 --gpus 1 --steps 20 --warmup 5 --R 16 --frames 100 || exit 1
bash scripts/gpu_prof_r4.sh r4e_split --gpus 1 --steps 20 --warmup 5 --mode split || exit 1
