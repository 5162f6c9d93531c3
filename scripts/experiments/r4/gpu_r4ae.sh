# Round 4 session ae: non-temporal IQ loads in the frame_td_fft512.hip
# receivers and k_mrc_any (the r4ad profiles showed HBM traffic 1.31-1.37x
# algorithmic: the streamed IQ evicting the frame's channel estimates from
# L2).  Same-process A/B against lib "head" (plain loads).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4ae; mkdir -p $OUT
for cfg in "1536 200" "3072 100" "6144 50" "256 800" "512 400" "1200 100"; do
  set -- $cfg
  timeout -k 10 240 python scripts/abx.py --C $1 --R 64 --frames $2 --reps 4 --stage demod prod head \
    > $OUT/ab_c$1.jsonl 2> $OUT/ab_c$1.err || { tail $OUT/ab_c$1.err; exit 1; }
  echo "C=$1"; grep -v "^{" $OUT/ab_c$1.jsonl
done
