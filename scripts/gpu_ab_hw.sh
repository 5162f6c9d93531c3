set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/abhw_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab_mrc.py 1250 4 default OFDM_MRC_ALIGN=1 OFDM_MRC_HW=16 OFDM_MRC_HW=16,OFDM_MRC_ALIGN=1 > $OUT/ab.txt 2>&1
rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env OFDM_MRC_HW=16 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/p16.log 2>&1
rc=$?; tail -2 $OUT/p16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env OFDM_MRC_ALIGN=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pa.log 2>&1
rc=$?; tail -2 $OUT/pa.log; exit $rc
