set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5al
timeout -k 10 400 python -u -m pytest tests/test_demod_onelaunch_gpu.py -q -k many_small_frames --timeout 180 --timeout-method thread > gpurun_out/r5al/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r5al/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/r5/r1_conditioning.py > gpurun_out/r5al/conditioning.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5al/conditioning.txt; exit $rc
