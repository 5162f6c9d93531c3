# round 6 (f): ZF apply with row pitches (ofdm_zf_apply_ex): ZF GPU tests, same-process layouts A/B at U = 16 / 32
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r6f; mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_zf_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for U in 16 32; do
  timeout -k 10 200 python3 scripts/zf_pitch_ab.py --op apply --U $U > $OUT/ab_apply_u$U.jsonl 2> $OUT/ab_apply_u$U.err || { tail $OUT/ab_apply_u$U.err; exit 1; }
  cat $OUT/ab_apply_u$U.jsonl
done
