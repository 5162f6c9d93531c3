# Round 4 session af: the receivers' HBM traffic after the non-temporal IQ
# loads (driver-form profiles, trace + PMC).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/gpu_prof_r4.sh r4af_c1536 --gpus 1 --steps 10 --warmup 3 --R 64 --C 1536 --frames 200 || exit 1
bash scripts/gpu_prof_r4.sh r4af_c6144 --gpus 1 --steps 10 --warmup 3 --R 64 --C 6144 --frames 50 || exit 1
bash scripts/gpu_prof_r4.sh r4af_c256 --gpus 1 --steps 10 --warmup 3 --R 64 --C 256 --frames 800 || exit 1
