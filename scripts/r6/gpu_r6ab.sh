# round 6 (ab): C = 3072 / 6144 receivers without their epilogue spill (lane recomputed in the epilogue) = prod vs
# pre (HEAD): any-C tests, A/B at R = 64 (3072 x 200 frames, 6144 x 100), headline unchanged check
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6ab; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_any_c_gpu.py tests/test_demod_onelaunch_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 3072 --R 64 --frames 200 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c3072.jsonl 2> $OUT/ab_c3072.err || { tail $OUT/ab_c3072.err; exit 1; }
tail -2 $OUT/ab_c3072.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 6144 --R 64 --frames 100 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c6144.jsonl 2> $OUT/ab_c6144.err || { tail $OUT/ab_c6144.err; exit 1; }
tail -2 $OUT/ab_c6144.jsonl
