set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5ai
timeout -k 10 600 python -u -m pytest tests/test_antenna_split_gpu.py -q -k "gpus2 or rccl_world1" --timeout 300 --timeout-method thread > gpurun_out/r5ai/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r5ai/pytest.log; exit $rc
