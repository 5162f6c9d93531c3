set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r4r
timeout -k 10 120 python scripts/fft_any_diag.py 1536 > gpurun_out/r4r/prod.txt 2>&1 && \
OFDM_LSMRC_LIB=diag timeout -k 10 120 python scripts/fft_any_diag.py 1536 > gpurun_out/r4r/diag.txt 2>&1
tail -3 gpurun_out/r4r/prod.txt; grep -v "^DIAG" gpurun_out/r4r/diag.txt | tail -2; grep "^DIAG" gpurun_out/r4r/diag.txt | tail -12
