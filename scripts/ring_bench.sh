#!/usr/bin/env bash
# Ingest rate through the ShMemSymBuff ring at the
# headline shape (R=64, C=1024, S=101 = one frame per ring): a writer process
# pushes NF frames (WithWait), the reader drains them with
#   frames:     gpuLS::demodFrames (pipelined bulk reader + ofdm_pipeline)
#   symbolcuda: the reference's per-symbol flow (readNextSymbolCUDA +
#               demodOneSymbol), one frame
# usage: bash scripts/ring_bench.sh [NF] [R] [C]   (outputs under gpurun_out/ring/)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
NF=${1:-100}; R=${2:-64}; C=${3:-1024}; S=101
OUT=$ROOT/gpurun_out/ring; mkdir -p $OUT; cd $OUT
PKG=$ROOT/gpu-accel-ofdm-ls-mrc_amd
for n in e2e_writer e2e_reader; do
  g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$PKG/host -I$ROOT/include \
    -DnumOfRows=$R -Ddimension=$C -Dprefix=0 -DlenOfBuffer=$S -DshmemID="\"/ofdm_ringbench_$$\"" \
    $ROOT/tests/cpp/$n.cpp -o $n -L$PKG/lib -lofdm_lsmrc -Wl,-rpath,$PKG/lib -L/opt/rocm/lib -lamdhip64 -lrt || exit 1
done
python3 - $R $C $S <<'PY' || exit 1
import sys, numpy as np
R, C, S = map(int, sys.argv[1:])
rng = np.random.default_rng(0)
K = C - 1
a = np.float32(0.70710678)
(rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64).tofile("Pilots.dat")
(rng.standard_normal((S, R, C)) + 1j * rng.standard_normal((S, R, C))).astype(np.complex64).tofile("iq.bin")
PY
for mode in "frames $NF 4 3" "frames $NF 1 3" "symbolcuda"; do
  set -- $mode
  rep=1; [ "$1" = frames ] && rep=$NF
  ./e2e_writer iq.bin $rep > writer.log 2>&1 &
  wpid=$!
  timeout -k 10 300 ./e2e_reader $mode > reader.json 2> reader.err
  rc=$?
  wait $wpid
  echo "$mode: rc=$rc $(cat reader.json)"
  [ $rc -eq 0 ] || exit $rc
done
