# round 6 (d): C = 2048 receiver with the 16-B transpose reads (prod) vs before (pc)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "2048" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/abx.py --C 2048 --R 64 --frames 400 --reps 6 --launches 5 --stage combine prod pc > $OUT/ab_c2k.jsonl 2> $OUT/ab_c2k.err || { tail $OUT/ab_c2k.err; exit 1; }
tail -2 $OUT/ab_c2k.jsonl
timeout -k 10 200 python -u scripts/abx.py --C 2048 --R 16 --frames 200 --reps 6 --launches 10 --stage combine prod pc > $OUT/ab_c2k_r16.jsonl 2> $OUT/ab_c2k_r16.err || { tail $OUT/ab_c2k_r16.err; exit 1; }
tail -2 $OUT/ab_c2k_r16.jsonl
