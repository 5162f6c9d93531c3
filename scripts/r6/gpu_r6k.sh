# round 6 (k): wave-uniform ticket code + quarter units at the one-launch demod's tail (prod: last k0/2 blocks
# quarters, k0/2 halves) vs qs0 (new ticket code, halves only = round-5 schedule) vs qs2 (k0/4 quarters, 3k0/4
# halves) vs pre (HEAD): tests, A/B at configs[1], headline, C = 2048 / 4096
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_demod_onelaunch_gpu.py tests/test_gpu_parity.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --reps 11 --launches 20 --stage demod prod qs0 qs2 pre > $OUT/ab_cfg1.jsonl 2> $OUT/ab_cfg1.err || { tail $OUT/ab_cfg1.err; exit 1; }
tail -4 $OUT/ab_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --reps 5 --launches 5 --stage demod prod qs0 pre > $OUT/ab_head.jsonl 2> $OUT/ab_head.err || { tail $OUT/ab_head.err; exit 1; }
tail -3 $OUT/ab_head.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c4k.jsonl 2> $OUT/ab_c4k.err || { tail $OUT/ab_c4k.err; exit 1; }
tail -2 $OUT/ab_c4k.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 2048 --R 64 --frames 400 --reps 5 --launches 5 --stage combine prod pre > $OUT/ab_c2k.jsonl 2> $OUT/ab_c2k.err || { tail $OUT/ab_c2k.err; exit 1; }
tail -2 $OUT/ab_c2k.jsonl
