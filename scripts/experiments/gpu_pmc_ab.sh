# PMC counters of the MRC kernel for a list of variants (ab_mrc.py workload).
# usage: [PMC_SETS="A B;C D"] [AB_FRAMES=400] bash scripts/experiments/gpu_pmc_ab.sh <tag> default VAR=VAL[,..] ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcab_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SETS=${PMC_SETS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"}
i=0
for v in "$@"; do
  IFS=';' read -ra PS <<< "$SETS"
  for P in "${PS[@]}"; do
    i=$((i+1))
    env $( [ "$v" = default ] || echo $v | tr ',' ' ' ) timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_mrc.py ${AB_FRAMES:-400} 1 default > $OUT/p$i.txt 2>&1
    rc=$?; echo "$v [$P] rc=$rc"; [ $rc -lt 124 ] || exit $rc
    [ $rc -eq 0 ] || { tail -3 $OUT/p$i.txt; continue; }
    python3 - $OUT/p$i/run_counter_collection.csv <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_mrc_td" in r["Kernel_Name"]]
agg = collections.defaultdict(list)
for r in rows: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("   ", {k: f"{sum(v)/len(v):.4g}" for k, v in agg.items()}, "launches", len(rows)//max(1,len(agg)))
PY
  done
done
