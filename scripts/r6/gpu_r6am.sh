# round 6 (am): antenna-split finalize without 64-bit divisions per element: split tests, then bench --mode split
# with the HEAD library (OFDM_LSMRC_LIB=pre) and the product, twice each alternately (stages_ms.finalize)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6am; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_antenna_split_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
OFDM_LSMRC_LIB=pre timeout -k 10 300 python -u bench.py --mode split --no-cpu --steps 20 --warmup 3 > $OUT/split_pre_$rep.json 2> $OUT/split_pre_$rep.err || { tail $OUT/split_pre_$rep.err; exit 1; }
timeout -k 10 300 python -u bench.py --mode split --no-cpu --steps 20 --warmup 3 > $OUT/split_prod_$rep.json 2> $OUT/split_prod_$rep.err || { tail $OUT/split_prod_$rep.err; exit 1; }
done
for f in $OUT/split_*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1]); st=d['stages_ms']
print('$f', round(d['ms_per_step'],3), 'finalize', round(st['finalize'],3), 'mrc', round(st['mrc_partial'],3), d['check']['vs_full_receiver']['ok'])"; done
