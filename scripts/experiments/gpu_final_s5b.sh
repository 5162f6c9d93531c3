#!/bin/bash
# Session-5 closing run: full GPU suite, smoke(), default bench, then the
# configs[2] (C=2048) bench line and profile of the final C=2048 receiver.
set -e -o pipefail
mkdir -p gpurun_out/s5 gpurun_out/pk2k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5/gpu_suite.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s5/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/s5/bench.json 2> gpurun_out/s5/bench.err
timeout -k 10 300 python -u bench.py --C 2048 --R 64 --frames 1000 --no-cpu --no-mode-a > gpurun_out/pk2k/bench.json 2> gpurun_out/pk2k/bench.err
bash scripts/experiments/gpu_prof_cfg.sh r2h_c2048 --C 2048 --R 64 --frames 1000 > gpurun_out/pk2k/prof.txt 2>&1
