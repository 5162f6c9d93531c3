# Round 4 session ac: occupancy A/B of the 512 / 256 / 128 receivers: product
# (114 / 106 / 102 VGPRs, 4 waves per SIMD) vs amdgpu_waves_per_eu 5 (96 VGPRs,
# 76 / 44 / 20 B of scratch) and 6 (80 VGPRs, 156 / 124 / 92 B), grids 5 / 6 per CU.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4ac; mkdir -p $OUT
for cfg in "512 400" "256 800" "128 1600"; do
  set -- $cfg
  timeout -k 10 240 python scripts/abx.py --C $1 --R 64 --frames $2 --reps 4 --stage demod prod occ5 occ6 \
    > $OUT/ab_c$1.jsonl 2> $OUT/ab_c$1.err || { tail $OUT/ab_c$1.err; exit 1; }
  grep -v "^{" $OUT/ab_c$1.jsonl
done
