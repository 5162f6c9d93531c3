# SQ counters of the headline MRC kernel (two passes, 8 SQ counters each).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sq_${1:-x}; mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py --frames 300 --steps 2 --warmup 1 --no-cpu > $OUT/p$i.json 2> $OUT/p$i.err
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
