# k_mrc_td1024_rsplit: parity tests, then same-process A/B vs the HLDS kernel
# at the configs[1] shape (R=16, 10k symbols) and the headline shape.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/rsplit_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rsplit or synth_vs_oracle or antenna_split" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
AB_R=16 timeout -k 10 200 python -u scripts/ab_mrc.py 100 5 default OFDM_MRC_RSPLIT=1 > $OUT/ab_r16_f100.log 2>&1 || exit 1
cat $OUT/ab_r16_f100.log
AB_R=16 timeout -k 10 200 python -u scripts/ab_mrc.py 1250 3 default OFDM_MRC_RSPLIT=1 > $OUT/ab_r16_f1250.log 2>&1 || exit 1
cat $OUT/ab_r16_f1250.log
timeout -k 10 200 python -u scripts/ab_mrc.py 100 5 default OFDM_MRC_RSPLIT=1 > $OUT/ab_r64_f100.log 2>&1 || exit 1
cat $OUT/ab_r64_f100.log
timeout -k 10 200 python -u scripts/ab_mrc.py 400 3 default OFDM_MRC_RSPLIT=1 > $OUT/ab_r64_f400.log 2>&1 || exit 1
cat $OUT/ab_r64_f400.log
