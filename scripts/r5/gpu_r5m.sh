# C = 4096 half units at the schedule tail (h4) vs product: configs[4] slice and the split mode's partial stage
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5m
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 400 --stage combine --reps 6 --launches 5 prod h4 h4z h4q > gpurun_out/r5m/abx_c4096.jsonl 2> gpurun_out/r5m/abx.err || exit 1; tail -2 gpurun_out/r5m/abx_c4096.jsonl
timeout -k 10 300 python -u scripts/abx.py --C 4096 --R 32 --frames 50 --stage partial --reps 6 --launches 8 prod h4 h4z h4q > gpurun_out/r5m/abx_partial50.jsonl 2>> gpurun_out/r5m/abx.err || exit 1; tail -2 gpurun_out/r5m/abx_partial50.jsonl
