# ZF GPU tests on the 16-B-store detect + A/B vs the r5g build
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5k
timeout -k 10 300 python -u -m pytest tests/test_zf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5k/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5k/pytest.log; [ $rc -eq 0 ] || exit $rc
for U in 8 16 32; do timeout -k 10 300 python -u scripts/zf_abx.py --U $U prod r5g > gpurun_out/r5k/zf_abx_u$U.jsonl 2> gpurun_out/r5k/zf_abx.err || exit 1; tail -2 gpurun_out/r5k/zf_abx_u$U.jsonl; done
