# one-launch demod: tables filled by waves 1-7 while wave 0 takes the ticket (f1) vs product; then the GPU suite on p1 is NOT run (A/B only)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5p
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --stage demod --reps 8 --launches 20 prod f1 > gpurun_out/r5p/abx_cfg1.jsonl 2> gpurun_out/r5p/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5p/abx_cfg1.jsonl | tail -2
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --stage demod --reps 4 --launches 5 prod f1 > gpurun_out/r5p/abx_default.jsonl 2>> gpurun_out/r5p/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5p/abx_default.jsonl | tail -2
