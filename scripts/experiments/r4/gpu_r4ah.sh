# Round 4 session ah: XCD-contiguous symbol spans in the 128..6144 receivers
# (each XCD walks one contiguous eighth of the data symbols, so a frame's
# estimate is fetched into one L2): parity tests, then same-process A/B
# against lib "head" (symbols round-robin over all XCDs).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r4ah; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_any_c_gpu.py tests/test_gpu_parity.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for cfg in "1536 200" "3072 100" "6144 50" "256 800" "512 400"; do
  set -- $cfg
  timeout -k 10 240 python scripts/abx.py --C $1 --R 64 --frames $2 --reps 4 --stage demod prod head \
    > $OUT/ab_c$1.jsonl 2> $OUT/ab_c$1.err || { tail $OUT/ab_c$1.err; exit 1; }
  echo "C=$1"; grep -v "^{" $OUT/ab_c$1.jsonl
done
