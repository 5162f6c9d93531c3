# Round 4 session l: PMC counters of the fused any-C MRC (k_mrc_any) at
# C = 1536, R = 64 (100 frames): where its time goes.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r4l}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--C ${C:-1536} --frames 100 --no-cpu --no-mode-a --steps 5 --warmup 2"
i=0
for ctr in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT/pmc$i" -o run \
    -- python3 "$ROOT/bench.py" $ARGS > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" || { tail -5 "$OUT/bench$i.err"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True)):
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_mrc_any" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[-3], {k: sum(x) / len(x) for k, x in v.items()})
PY
