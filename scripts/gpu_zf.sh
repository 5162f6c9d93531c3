set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/zf_${1:-x}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_zf_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "zf pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/zf_bench.py ${ZF_ARGS:---ab} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o zf -- python3 scripts/zf_bench.py --U 16 --no-cpu --reps 5 > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
for f in $(find $OUT/prof -name "*kernel_stats.csv"); do echo $f; cut -d, -f1-8 $f | head -12; done
exit $rc
