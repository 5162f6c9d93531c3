#!/usr/bin/env bash
# Default bench: warm-up 3 (default) vs 10 vs 20 untimed steps, alternating.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=gpurun_out/r3z5; mkdir -p $OUT
for rep in 1 2; do
  for w in 3 10 20; do
    timeout -k 10 200 python -u bench.py --no-cpu --no-mode-a --warmup $w > $OUT/w${w}_$rep.json 2> $OUT/w${w}_$rep.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,3), round(d['ms_per_step'],3), d['roofline']['median_launch_ms'])" $OUT/w${w}_$rep.json
  done
done
