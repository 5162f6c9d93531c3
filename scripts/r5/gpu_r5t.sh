# work tickets: one workspace shared by two batch geometries (r5g library, then the product), capture tests
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5t
OFDM_LSMRC_LIB=r5g timeout -k 10 300 python -u -m pytest tests/test_demod_onelaunch_gpu.py -q -k two_geometries --timeout 120 --timeout-method thread > gpurun_out/r5t/old.log 2>&1; rc=$?
echo "r5g library rc=$rc"; tail -3 gpurun_out/r5t/old.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5t/new.log 2>&1; rc=$?
echo "product rc=$rc"; tail -3 gpurun_out/r5t/new.log; exit $rc
