set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5aa
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5aa/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r5aa/pytest.log; exit $rc
