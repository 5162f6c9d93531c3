# round 6 (ac): generic any-C path with a non-hoistable thread index (k_mrc_any 260-296 -> 0 B of scratch,
# k_fft_any 106-166 -> 66-84 VGPRs) = prod vs pre (HEAD): any-C tests, A/B at C = 1200 / 2400 / 5000
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6ac; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_any_c_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for c in 1200 2400 5000; do
timeout -k 10 300 python -u scripts/abx.py --C $c --R 64 --frames 50 --reps 5 --launches 3 --stage combine prod pre > $OUT/ab_c$c.jsonl 2> $OUT/ab_c$c.err || { tail $OUT/ab_c$c.err; exit 1; }
tail -2 $OUT/ab_c$c.jsonl
done
