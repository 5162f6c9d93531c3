# one-launch demod: half units for the last k0 (product), 2 k0, 4 k0 blocks per range, or all blocks
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5ae
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --stage demod --reps 8 --launches 20 prod s2 s4 sall > gpurun_out/r5ae/abx_cfg1.jsonl 2> gpurun_out/r5ae/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5ae/abx_cfg1.jsonl | tail -4
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --stage demod --reps 4 --launches 5 prod s2 s4 > gpurun_out/r5ae/abx_default.jsonl 2>> gpurun_out/r5ae/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5ae/abx_default.jsonl | tail -3
