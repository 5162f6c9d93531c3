# split pipeline with one batch LS (ofdm_frame_mrc_partial_range): split GPU tests, then bench --mode split (stage times)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest tests/test_antenna_split_gpu.py -q --timeout 180 --timeout-method thread > gpurun_out/r5v/pytest.log 2>&1; rc=$?
echo "split tests rc=$rc"; tail -3 gpurun_out/r5v/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode split --no-cpu > gpurun_out/r5v/bench_split.json 2> gpurun_out/r5v/bench_split.err; rc=$?
echo "split bench rc=$rc"; tail -c 2500 gpurun_out/r5v/bench_split.json; exit $rc
