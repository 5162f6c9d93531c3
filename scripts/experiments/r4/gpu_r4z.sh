# Round 4 closing evidence: GPU suite and smoke on the final product library,
# then the driver-form profile of the default bench (un-profiled, kernel
# trace, PMC passes) and of the C = 4096 slice.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4z; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash scripts/gpu_prof_r4.sh r4z || exit 1
bash scripts/gpu_prof_r4.sh r4z_c4096 --gpus 1 --steps 20 --warmup 5 --R 32 --C 4096 --frames 400 || exit 1
