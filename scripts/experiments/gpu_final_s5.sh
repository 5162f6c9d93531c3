#!/bin/bash
# Session-5 final tree: full GPU suite, smoke(), default bench line.
set -e -o pipefail
mkdir -p gpurun_out/s5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5/gpu_suite.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s5/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/s5/bench.json 2> gpurun_out/s5/bench.err
