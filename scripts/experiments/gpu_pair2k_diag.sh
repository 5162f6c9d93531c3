#!/usr/bin/env bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/pair2k; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "2048 and not 1000" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 64 --frames 200 --reps 3 default MRC2KP_DBG=1 MRC2KP_DBG=64 MRC2KP_XCH=1 MRC2K_PAIR=0 > $OUT/diag2.jsonl 2>&1; rc=$?; cut -c1-150 $OUT/diag2.jsonl; exit $rc
