set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -30 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; echo "bench rc=$?"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
