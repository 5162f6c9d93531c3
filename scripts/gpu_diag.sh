cd $GRAFT_REPO_ROOT
OUT=gpurun_out/diag_$1; mkdir -p $OUT
for v in default OFDM_MRC_DEBUG=1 OFDM_MRC_DEBUG=2 OFDM_MRC_DEBUG=3; do
  env $( [ "$v" = default ] || echo $v ) timeout -k 10 200 python bench.py --frames 1250 --steps 10 --warmup 2 --no-cpu > $OUT/b.json 2> $OUT/b.err
  rc=$?; python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$v', round(d['roofline']['avg_launch_ms'],3), 'ms', round(d['roofline']['achieved']), 'GB/s', round(d['roofline']['frac'],3))" || echo "$v rc=$rc"
  [ $rc -lt 124 ] || exit $rc
done
