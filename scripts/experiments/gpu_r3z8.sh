#!/usr/bin/env bash
# ZF detect (k_zf_wstat): symbol quads per wave step SG = 4 (default, PD 2)
# vs SG = 2 with PD 2 (ZF_LDS=15) / PD 4 (ZF_LDS=16), U = 16 and 32.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3z8; mkdir -p $OUT
for U in 16 32; do
  timeout -k 10 200 python -u scripts/zf_ab.py --U $U --reps 10 default ZF_LDS=15 ZF_LDS=16 >> $OUT/ab.jsonl 2> $OUT/ab_$U.err || exit 1
done
python -c "import sys,json; [print(d['variant'],d['U'],d['detect_ms'],d['detect_frac'],d['max_rel_diff_vs_first']) for d in map(json.loads,open(sys.argv[1]))]" $OUT/ab.jsonl
