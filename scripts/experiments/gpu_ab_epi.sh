#!/usr/bin/env bash
# GPU parity suite, then same-process A/B of the staged nontemporal output
# epilogues against the round-1 scattered-store epilogues (C=2048 bit 3,
# C=4096 bit 5) and the C=1024 plain-store variant (bit 5).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/abepi_${1:-x}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u scripts/ab.py --C 1024 --R 64 --frames 400 --reps 4 default MRC1K_DBG=32 \
  > $OUT/c1024.jsonl 2> $OUT/c1024.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 2048 --R 64 --frames 200 --reps 4 default MRC2K_DBG=8 \
  > $OUT/c2048.jsonl 2> $OUT/c2048.err || exit 1
timeout -k 10 300 python -u scripts/ab.py --C 4096 --R 32 --frames 300 --reps 4 default MRC4K_DBG=32 \
  > $OUT/c4096.jsonl 2> $OUT/c4096.err || exit 1
cat $OUT/*.jsonl
