# round 6 (b): tagged tickets claimed by workgroup 0 (prod) vs compare-and-swap claims only (tk) vs round 5 (r5)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod tk r5 > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -3 $OUT/ab_cfg1.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod r5 > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -2 $OUT/ab_head.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine prod r5 > $OUT/ab_c4k.jsonl 2> $OUT/ab_c4k.err || { tail $OUT/ab_c4k.err; exit 1; }
tail -2 $OUT/ab_c4k.jsonl
