#!/usr/bin/env bash
# Effective shader clock of MRC kernel variants: GRBM_GUI_ACTIVE (GPU clock
# cycles while busy) over the dispatch's kernel-trace duration.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=$1; C=$2; R=$3; FR=$4; shift 4
OUT=gpurun_out/clk_$TAG; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE --output-format csv -d $OUT/p -o run -- \
  python3 scripts/ab.py --C $C --R $R --frames $FR --reps 1 "$@" > $OUT/ab.jsonl 2> $OUT/ab.err || exit 1
python3 scripts/experiments/clock_table.py $OUT/p
