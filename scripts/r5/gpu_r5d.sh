set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5f
timeout -k 10 400 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5f/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_session.sh r5f abx:--C:1024:--R:16:--frames:100:--stage:demod:--reps:6:--launches:20:prod:s2:nopf:tk abx:--C:1024:--R:64:--frames:1250:--stage:demod:--reps:4:--launches:5:prod:s2:nopf:tk cfg1 c4096 default
