# round 6 (ap): PN sync GPU tests on the build with the 32-bit extract, then the final profiles
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6ap; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_pn_sync_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash scripts/gpu_session.sh r6ap prof_default prof_cfg1 prof_c4096 prof_split
