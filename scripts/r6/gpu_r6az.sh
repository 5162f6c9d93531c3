# round 6 (az): reciprocal normalisation in mode A (k_mrc_freq*), the generic any-C receiver, the MFMA combine
# and the split finalize (prod) vs pre (HEAD): GPU suite, bench --mode freq alternating, generic A/B at C = 1200
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6az; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
OFDM_LSMRC_LIB=pre timeout -k 10 300 python -u bench.py --mode freq --no-cpu --steps 20 --warmup 3 > $OUT/freq_pre_$rep.json 2> $OUT/freq_pre_$rep.err || { tail $OUT/freq_pre_$rep.err; exit 1; }
timeout -k 10 300 python -u bench.py --mode freq --no-cpu --steps 20 --warmup 3 > $OUT/freq_prod_$rep.json 2> $OUT/freq_prod_$rep.err || { tail $OUT/freq_prod_$rep.err; exit 1; }
done
for f in $OUT/freq_*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['ms_per_step'],4), 'kernel', round(r['avg_launch_ms'],4), round(r['frac'],4))"; done
timeout -k 10 300 python -u scripts/abx.py --C 1200 --R 64 --frames 50 --reps 5 --launches 3 --stage combine prod pre > $OUT/ab_c1200.jsonl 2> $OUT/ab_c1200.err || { tail $OUT/ab_c1200.err; exit 1; }
tail -2 $OUT/ab_c1200.jsonl
