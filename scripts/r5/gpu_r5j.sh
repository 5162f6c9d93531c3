# ZF detect: line-aligned rows (K = 1024) vs K = 1023, product and 16-B stores
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5j
for K in 1024 1023; do timeout -k 10 300 python -u scripts/zf_abx.py --U 16 --K $K --rounds 4 prod zS16 zdbgC zdbgD > gpurun_out/r5j/zf_k$K.jsonl 2> gpurun_out/r5j/zf.err || exit 1; tail -4 gpurun_out/r5j/zf_k$K.jsonl; done
