#!/usr/bin/env bash
# Tail quantisation probe: one-launch C=1024 R=16 throughput vs batch size
# (MRC workgroups = 12.5 x frames at S=101; 512 resident at 2 per CU).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3x; mkdir -p $OUT
for F in 40 41 60 80 82 100 120 123 160 164 200 400; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-mode-a --R 16 --frames $F --steps 200 --warmup 20 > $OUT/f$F.json 2> $OUT/f$F.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value']/1e6, d['ms_per_step'], d['roofline']['frac'])" $OUT/f$F.json $F
done
