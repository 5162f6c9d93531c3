cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=$1; shift
if [ "$RUN_TESTS" = 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1; prc=$?; echo "pytest rc=$prc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $prc -lt 124 ] || exit $prc
fi
timeout -k 10 600 python scripts/ab_mrc.py ${AB_F:-1250} 3 "$@" > gpurun_out/ab_$TAG.txt 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/ab_$TAG.txt
if [ "$RUN_PROBE" = 1 ]; then timeout -k 10 120 ./scripts/bwprobe2 > gpurun_out/bwprobe2_$TAG.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/bwprobe2_$TAG.txt; fi
