# C = 4096: twiddles from LDS tables (t4TT: both stages; t4TA: stage A only) vs anchors (product)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5n
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --stage combine --reps 6 --launches 5 prod t4TT t4TA > gpurun_out/r5n/abx_c4096.jsonl 2> gpurun_out/r5n/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5n/abx_c4096.jsonl | tail -3
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 50 --stage partial --reps 6 --launches 8 prod t4TT t4TA > gpurun_out/r5n/abx_partial50.jsonl 2>> gpurun_out/r5n/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5n/abx_partial50.jsonl | tail -3
