# scratch-size artifact check: the same A/B with 200 launches per rep (a per-switch scratch reallocation amortised),
# then each library in its own bench process (configs[1], 200 steps after 50 warm-up steps)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5ah
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --stage demod --reps 6 --launches 200 prod ni0 ni1 > gpurun_out/r5ah/abx_cfg1_l200.jsonl 2> gpurun_out/r5ah/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5ah/abx_cfg1_l200.jsonl | tail -3
for lib in prod ni0 ni1 prod; do
  if [ $lib = prod ]; then L=""; else L=$lib; fi
  OFDM_LSMRC_LIB=$L timeout -k 10 200 python -u bench.py --R 16 --frames 100 --steps 200 --warmup 50 --no-cpu --no-box > gpurun_out/r5ah/bench_$lib.json 2> gpurun_out/r5ah/bench.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ah/bench_$lib.json').read().strip().splitlines()[-1]); print('$lib', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done
