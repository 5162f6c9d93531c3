# A/B the MRC row-loop variants + SQ counters on one box.
# usage: bash scripts/gpu_variants.sh <tag>
cd $GRAFT_REPO_ROOT
TAG=${1:-v}
OUT=gpurun_out/var_$TAG; mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --frames 500 --steps 10 --warmup 2 --no-cpu > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', round(d['roofline']['avg_launch_ms'],3), 'ms', round(d['roofline']['frac'],3), 'frac', d['check'])" 2>/dev/null || echo "$name failed rc=$rc"
  [ $rc -lt 124 ] || exit $rc
}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest.log 2>&1; prc=$?; echo "pytest rc=$prc"; tail -3 $OUT/pytest.log
[ $prc -lt 124 ] || exit $prc
for w in 4 8; do for sc in 1 0; do run w${w}_s${sc} OFDM_MRC_WAVES=$w OFDM_MRC_SCHED=$sc; done; done
run w8_s1_nt0 OFDM_MRC_WAVES=8 OFDM_MRC_SCHED=1 OFDM_MRC_NT=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$OUT/counters.txt 2>&1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $P --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --frames 200 --steps 1 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$OUT/pmc$i.json 2> $GRAFT_REPO_ROOT/$OUT/pmc$i.err
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -lt 124 ] || exit $rc
done
echo done
