# Round 4: same-process library A/B (scripts/abx.py) at C = 4096: prod vs ea
# (next row's first quarter issued at the row start)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r4d}; mkdir -p $OUT
for spec in "combine 300" "combine 400" "partial 400"; do
  set -- $spec
  timeout -k 10 300 python scripts/abx.py --stage $1 --C 4096 --R 32 --frames $2 --reps 4 prod ea > $OUT/abx_${1}_$2.jsonl 2>&1 || { tail $OUT/abx_${1}_$2.jsonl; exit 1; }
  tail -2 $OUT/abx_${1}_$2.jsonl
done
