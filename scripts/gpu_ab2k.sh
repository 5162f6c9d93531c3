set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab2k_${1:-x}; shift; mkdir -p $OUT
V=${PARITY_VAR:-OFDM_MRC2K_H=4}
timeout -k 10 300 env $V python -u -m pytest tests/test_gpu_parity.py tests/test_antenna_split_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/p.log 2>&1
rc=$?; tail -3 $OUT/p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env AB_C=2048 AB_R=64 python -u scripts/ab_mrc.py 400 3 "$@" > $OUT/ab.txt 2>&1
rc=$?; cat $OUT/ab.txt; exit $rc
