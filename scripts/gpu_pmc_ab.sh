# PMC counters of the MRC kernel for a list of variants (ab_mrc.py workload)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcab_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  for P in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
    i=$((i+1))
    env $( [ "$v" = default ] || echo $v | tr ',' ' ' ) timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_mrc.py 400 1 default > $OUT/p$i.txt 2>&1
    rc=$?; echo "$v [$P] rc=$rc"; [ $rc -lt 124 ] || exit $rc
    python3 - $OUT/p$i/run_counter_collection.csv <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mrc_td1024" in r["Kernel_Name"]]
agg = collections.defaultdict(list)
for r in rows: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("   ", {k: f"{sum(v)/len(v):.4g}" for k, v in agg.items()}, "launches", len(rows)//max(1,len(agg)))
PY
  done
done
