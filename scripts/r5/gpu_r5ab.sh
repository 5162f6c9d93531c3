# pipeline with ticketed chunks and a short tail (the product library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r5ab


timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5ab/new.log 2>&1; rc=$?
echo "product rc=$rc"; tail -2 gpurun_out/r5ab/new.log; exit $rc
