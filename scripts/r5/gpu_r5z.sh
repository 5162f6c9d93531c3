# ZF evidence (round 5): GPU tests, bench line at U = 16, rocprof trace, PMC passes (FETCH_SIZE; WRITE_SIZE;
# GRBM_GUI_ACTIVE + SQ), each its own run; summarised by scripts/zf_prof_summary.py
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r5z; mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_zf_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $ROOT/scripts/zf_bench.py --U 16 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/scripts/zf_bench.py --U 16 --no-cpu --reps 5 > $OUT/bench_trace.json 2> $OUT/bench_trace.err || { tail $OUT/bench_trace.err; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"; do
  name=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $OUT/pmc_$name -o run -- python3 $ROOT/scripts/zf_bench.py --U 16 --no-cpu --reps 3 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
done
echo "r5z done"
