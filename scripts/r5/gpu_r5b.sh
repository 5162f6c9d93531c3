set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5c
timeout -k 10 400 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_gpu_parity.py tests/test_e2e_gpu.py tests/test_antenna_split_gpu.py tests/test_any_c_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5c/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_session.sh r5c abx:--C:1024:--R:64:--frames:1250:--stage:demod:--reps:4:--launches:5:prod:r5base:ns:cas abx:--C:1024:--R:16:--frames:100:--stage:demod:--reps:6:--launches:20:prod:r5base:ns:cas abx:--C:4096:--R:32:--frames:400:--stage:combine:--reps:4:--launches:5:prod:r5base abx:--C:2048:--R:64:--frames:400:--stage:combine:--reps:4:--launches:5:prod:r5base
