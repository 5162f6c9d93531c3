# configs[2] (R=64, C=2048, 1000 frames): fused line with stamps, and the frequency-domain (mode A) line on the same box
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5y
timeout -k 10 300 python -u bench.py --R 64 --C 2048 --frames 1000 --steps 10 --warmup 3 --no-cpu --stamps-out gpurun_out/r5y/stamps_cfg2.npy > gpurun_out/r5y/cfg2.json 2> gpurun_out/r5y/cfg2.err || exit 1
timeout -k 10 300 python -u bench.py --mode freq --R 64 --C 2048 --frames 1000 --steps 10 --warmup 3 --no-cpu > gpurun_out/r5y/cfg2_freq.json 2> gpurun_out/r5y/cfg2_freq.err || exit 1
for f in cfg2 cfg2_freq; do python3 -c "import json; d=json.loads(open('gpurun_out/r5y/$f.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(d['ms_per_step'],3), round(r['frac'],4), r.get('avg_launch_ms'))"; done
