# the host-ingest pipeline with ticketed chunks and a short tail on the build before the ticket fixes (r5g) and on the product
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5ak
OFDM_LSMRC_LIB=r5g timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -q -k short_tail --timeout 120 --timeout-method thread > gpurun_out/r5ak/old.log 2>&1; rc=$?
echo "r5g rc=$rc"; tail -2 gpurun_out/r5ak/old.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -q -k short_tail --timeout 120 --timeout-method thread > gpurun_out/r5ak/new.log 2>&1; rc=$?
echo "product rc=$rc"; tail -2 gpurun_out/r5ak/new.log; exit $rc
