# C = 1024 receivers' shared-row loop with packed-f32 FFT halves (pkb2: second half; pkab: both) vs product
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5aj
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --stage demod --reps 8 --launches 20 prod pkb2 pkab > gpurun_out/r5aj/abx_cfg1.jsonl 2> gpurun_out/r5aj/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5aj/abx_cfg1.jsonl | tail -3
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --stage demod --reps 4 --launches 5 prod pkb2 pkab > gpurun_out/r5aj/abx_default.jsonl 2>> gpurun_out/r5aj/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5aj/abx_default.jsonl | tail -3
