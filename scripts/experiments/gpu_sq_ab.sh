#!/usr/bin/env bash
# SQ counters (two passes, 8 SQ counters each) of MRC kernel variants from the
# A/B build, one short ab.py run per pass: scripts/experiments/gpu_sq_ab.sh <tag> <C> <R> <variants...>
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=$1; C=$2; R=$3; shift 3
OUT=gpurun_out/sqab_$TAG; mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- \
    python3 scripts/ab.py --C $C --R $R --frames 100 --reps 1 "$@" > $OUT/p$i.jsonl 2> $OUT/p$i.err
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/experiments/sq_table.py $OUT
