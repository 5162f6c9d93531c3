#!/usr/bin/env bash
# FETCH_SIZE calibration for the ZF apply access pattern: plain vs nontemporal
# input loads of the same kernel (same bytes), raw KiB per dispatch.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/zfcal_${1:-x}; mkdir -p $OUT
for V in default ZF_NT=1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_${V/=/} -o run -- \
    python3 scripts/zf_ab.py --U 16 --nsym 4000 --reps 1 $V > /dev/null 2> $OUT/pmc_${V/=/}.err || exit 1
done
echo done
