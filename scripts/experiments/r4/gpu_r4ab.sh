# Round 4 session ab: the C = 128 / 256 receivers (k_mrc_td128 / k_mrc_td256,
# NR antenna rows per wave pass, templated with 512): parity, then same-process
# A/B against the previous library (lib "head": 512 on the old td512 kernel,
# 256 / 128 on the generic k_mrc_any).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_any_c_gpu.py tests/test_gpu_parity.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
for cfg in "512 400" "256 800" "128 1600"; do
  set -- $cfg
  timeout -k 10 240 python scripts/abx.py --C $1 --R 64 --frames $2 --reps 4 --stage demod prod head \
    > $OUT/ab_c$1.jsonl 2> $OUT/ab_c$1.err || { tail $OUT/ab_c$1.err; exit 1; }
  grep -v "^{" $OUT/ab_c$1.jsonl
done
