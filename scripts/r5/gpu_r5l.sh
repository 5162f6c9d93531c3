# estimator: first row loads before the table fill + next row prefetched (est2) vs product
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5l
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --stage demod --reps 8 --launches 20 prod est2 > gpurun_out/r5l/abx_cfg1.jsonl 2> gpurun_out/r5l/abx.err || exit 1; tail -2 gpurun_out/r5l/abx_cfg1.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --stage demod --reps 4 --launches 5 prod est2 > gpurun_out/r5l/abx_default.jsonl 2>> gpurun_out/r5l/abx.err || exit 1; tail -2 gpurun_out/r5l/abx_default.jsonl
