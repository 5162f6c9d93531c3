# ZF detect bytes with 32-subcarrier x 8-row tiles (probe zp32, 256-B pieces) vs the 16-subcarrier probe (zdbgC) and the product
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5q
for K in 1023 1024; do timeout -k 10 300 python -u scripts/zf_abx.py --U 16 --K $K --rounds 4 prod zdbgC zp32 > gpurun_out/r5q/zf_k$K.jsonl 2> gpurun_out/r5q/zf.err || exit 1; tail -3 gpurun_out/r5q/zf_k$K.jsonl; done
