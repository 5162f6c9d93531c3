# Round 4 session ad: driver-form profiles (trace + PMC wave-state counters)
# of the wave-pair (C = 3072) and wave-quad (C = 6144) receivers.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/gpu_prof_r4.sh r4ad_c3072 --gpus 1 --steps 10 --warmup 3 --R 64 --C 3072 --frames 100 || exit 1
bash scripts/gpu_prof_r4.sh r4ad_c6144 --gpus 1 --steps 10 --warmup 3 --R 64 --C 6144 --frames 50 || exit 1
bash scripts/gpu_prof_r4.sh r4ad_c1536 --gpus 1 --steps 10 --warmup 3 --R 64 --C 1536 --frames 200 || exit 1
