cd $GRAFT_REPO_ROOT
OUT=gpurun_out/quick_$1; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest.log 2>&1; prc=$?; echo "pytest rc=$prc"; tail -4 $OUT/pytest.log
[ $prc -lt 124 ] || exit $prc
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/b.json 2> $OUT/b.err
rc=$?; python3 -c "import json; d=json.load(open('$OUT/b.json')); print(round(d['value']/1e6,3),'M sym/s', round(d['roofline']['avg_launch_ms'],3), 'ms', round(d['roofline']['achieved']), 'GB/s', round(d['roofline']['frac'],3), d['stages_ms'], d['check'])" || echo "bench rc=$rc"
