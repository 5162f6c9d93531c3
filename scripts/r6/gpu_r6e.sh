# round 6 (e): ZF detect with row pitches (ofdm_zf_detect_ex): ZF GPU tests, same-process layouts A/B at U = 16 / 32,
# rocprof kernel trace + PMC of the padded and reference layouts
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r6e; mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_zf_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 scripts/zf_pitch_ab.py --U 16 > $OUT/ab_u16.jsonl 2> $OUT/ab_u16.err || { tail $OUT/ab_u16.err; exit 1; }
cat $OUT/ab_u16.jsonl
timeout -k 10 200 python3 scripts/zf_pitch_ab.py --U 32 > $OUT/ab_u32.jsonl 2> $OUT/ab_u32.err || { tail $OUT/ab_u32.err; exit 1; }
cat $OUT/ab_u32.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/scripts/zf_pitch_ab.py --U 16 --reps 2 > $OUT/trace.jsonl 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o run -- python3 $ROOT/scripts/zf_pitch_ab.py --U 16 --reps 1 --launches 2 > $OUT/pmc_$ctr.jsonl 2> $OUT/pmc_$ctr.err || { tail $OUT/pmc_$ctr.err; exit 1; }
done
echo r6e done
