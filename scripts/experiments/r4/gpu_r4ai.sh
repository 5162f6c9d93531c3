# Round 4 session ai: one row-pointer division per data symbol (not per row) and a
# wave-uniform wave index in the 128..6144 receivers:
# parity tests, then same-process A/B
# against lib "head" (the per-row 64-bit division on the VALU).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4ai; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_any_c_gpu.py tests/test_gpu_parity.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for cfg in "1536 200" "3072 100" "6144 50" "256 800" "512 400" "128 1600"; do
  set -- $cfg
  timeout -k 10 240 python scripts/abx.py --C $1 --R 64 --frames $2 --reps 4 --stage demod prod head \
    > $OUT/ab_c$1.jsonl 2> $OUT/ab_c$1.err || { tail $OUT/ab_c$1.err; exit 1; }
  echo "C=$1"; grep -v "^{" $OUT/ab_c$1.jsonl
done
