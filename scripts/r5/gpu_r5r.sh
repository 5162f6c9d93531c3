# ZF detect with non-temporal input loads (zntl: the input stream no longer evicts the partially written output lines from L2) vs product
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5r
for U in 16 32; do timeout -k 10 300 python -u scripts/zf_abx.py --U $U --rounds 4 prod zntl > gpurun_out/r5r/zf_u$U.jsonl 2> gpurun_out/r5r/zf.err || exit 1; tail -2 gpurun_out/r5r/zf_u$U.jsonl; done
