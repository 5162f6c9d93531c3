# k_mrc_td2048_lr: the whole GPU parity + antenna-split suites with the
# variant forced (OFDM_MRC2K_LR=1 and 2), then the same-process A/B at
# configs[2]'s shape (R=64, C=2048; 400 frames).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/ab2k_lr_${1:-x}; mkdir -p $OUT
for v in 1 2; do
  OFDM_MRC2K_LR=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_antenna_split_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/p$v.log 2>&1
  rc=$?; tail -2 $OUT/p$v.log; [ $rc -eq 0 ] || exit $rc
done
AB_C=2048 AB_R=64 timeout -k 10 300 python -u scripts/ab_mrc.py 400 3 default OFDM_MRC2K_LR=1 OFDM_MRC2K_LR=2 > $OUT/ab.txt 2>&1
rc=$?; cat $OUT/ab.txt; exit $rc
