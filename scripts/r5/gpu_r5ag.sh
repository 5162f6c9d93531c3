# estimator as a non-inlined function (ni0: same code; ni1: + first row before the table fill, next row prefetched) vs product
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5ag
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 16 --frames 100 --stage demod --reps 8 --launches 20 prod ni0 ni1 > gpurun_out/r5ag/abx_cfg1.jsonl 2> gpurun_out/r5ag/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5ag/abx_cfg1.jsonl | tail -3
timeout -k 10 300 python -u scripts/abx.py --C 1024 --R 64 --frames 1250 --stage demod --reps 4 --launches 5 prod ni0 ni1 > gpurun_out/r5ag/abx_default.jsonl 2>> gpurun_out/r5ag/abx.err || exit 1; grep -v '"rep"' gpurun_out/r5ag/abx_default.jsonl | tail -3
