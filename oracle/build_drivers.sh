#!/usr/bin/env bash
# build_drivers.sh -- TEST INFRASTRUCTURE ONLY: build the reference's own
# drivers against this package's drop-in headers,
# for the end-to-end driver test (tests/test_ref_drivers.py).
#
# Read where they lie in /root/reference (nothing is copied into the repo):
#   cpuLS_main.cpp    unchanged (copied to a scratch directory), with
#                     INTEGRATION.md's g++ command;
#   gpuLS_main.cu     through host/port_cuda_driver.sed (the documented
#                     mechanical CUDA -> HIP edits), then the same command;
#   rx_and_corr.cpp   its ring-writer code -- lines 48-60 (ring header,
#                     mode, buffPtr, copy_buff, cp_size) and copy_to_shared_mem
#                     (64-87) -- unchanged, in front of oracle/rx_writer_harness.cpp
#                     (the UHD/boost radio loop around them is not buildable).
# One binary set per ring geometry (the ring is configured at compile time,
# as in the reference).  Output: oracle/_ref/drivers/ (git-ignored; built
# here, travels to the GPU box with the snapshot; rpath is $ORIGIN-relative).
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
PKG="$ROOT/gpu-accel-ofdm-ls-mrc_amd"
OUT="$HERE/_ref/drivers"
if [ ! -f "$REF/cpuLS_main.cpp" ]; then
  echo "build_drivers.sh: $REF not present; skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
CXX=(g++ -O2 -std=c++17 -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I"$PKG/host" -I"$ROOT/include")
LIBS=(-L"$PKG/lib" -lofdm_lsmrc '-Wl,-rpath,$ORIGIN/../../../gpu-accel-ofdm-ls-mrc_amd/lib' -L/opt/rocm/lib -lamdhip64 -lrt)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
# into a scratch directory: a quoted #include searches the source's own
# directory first, which must not be /root/reference (its headers are the
# ones being replaced)
cp "$REF/cpuLS_main.cpp" "$TMP/cpuLS_main.cpp"
sed -f "$PKG/host/port_cuda_driver.sed" "$REF/gpuLS_main.cu" > "$TMP/gpuLS_main.cpp"
{
  echo '#include <complex>'
  echo '#include <cstdio>'
  echo '#include <cstdlib>'
  echo '#include <cstring>'
  echo '#include <fstream>'
  echo '#include <vector>'
  awk '/#include "ShMemSymBuff_gpu.hpp"/ { on = 1 } /^namespace po/ { on = 0 } on' "$REF/rx_and_corr.cpp"
  awk '/^void copy_to_shared_mem\(/ { on = 1 } on { print } on && /^}/ { exit }' "$REF/rx_and_corr.cpp"
  cat "$HERE/rx_writer_harness.cpp"
} > "$TMP/rx_writer.cpp"
# geometry: R C S (the golden fixtures the test drives through them)
for g in "4 1024 10" "8 2048 3"; do
  set -- $g
  tag="r$1_c$2_s$3"
  D=(-DnumOfRows=$1 -Ddimension=$2 -Dprefix=0 -DlenOfBuffer=$3 "-DshmemID=\"/ofdm_refdrv_$tag\"")
  "${CXX[@]}" "${D[@]}" "$TMP/cpuLS_main.cpp" -o "$OUT/cpuLS_main_$tag" "${LIBS[@]}" 2> "$TMP/log" ||
    { cat "$TMP/log" >&2; exit 1; }
  "${CXX[@]}" "${D[@]}" "$TMP/gpuLS_main.cpp" -o "$OUT/gpuLS_main_$tag" "${LIBS[@]}"
  "${CXX[@]}" "${D[@]}" "$TMP/rx_writer.cpp" -o "$OUT/rx_writer_$tag" "${LIBS[@]}"
done
echo "built $OUT"
