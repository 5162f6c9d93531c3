# graph capture of the work-ticketed receivers (capture counter set behind a zeroing kernel node):
# the debug script (counters per replay), then the one-launch / ticket test file
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5s
timeout -k 10 120 python -u scripts/r5/capture_debug.py > gpurun_out/r5s/capture_debug.txt 2>&1 || { tail -5 gpurun_out/r5s/capture_debug.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5s/capture_debug.txt
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5s/new.log 2>&1; rc=$?
echo "product rc=$rc"; tail -3 gpurun_out/r5s/new.log; exit $rc
