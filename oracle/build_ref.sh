#!/usr/bin/env bash
# build_ref.sh -- compile the reference's own RX arithmetic into oracle/_ref/.
#
# TEST INFRASTRUCTURE ONLY.  The reference's cpuLS.hpp cannot be compiled as a
# whole here: it #includes <fftw3.h> and <cblas.h>, and FFTW3 / CBLAS / LAPACK
# are absent from the image (no stand-ins are written for them).  What this
# recipe does instead: pipe the FFT-free RX functions straight from
# /root/reference/cpuLS.hpp (read where they lie, nothing is copied into the
# repo or written to disk) into g++, behind the reference's own ShMemSymBuff.hpp
# for complexF, and link them with oracle/ref_harness.cpp.  Output:
# oracle/_ref/libref_cpuls.so (git-ignored; travels to the GPU box with the
# snapshot but is not needed there).
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -f "$REF/cpuLS.hpp" ]; then
  echo "build_ref.sh: $REF/cpuLS.hpp not present; skipping reference build" >&2
  exit 0
fi
mkdir -p "$OUT"
FUNCS="matrix_readX shiftOneRow matrixMultThenSum findDistSqrd divideOneRow rotCube"
{
  for f in $FUNCS; do
    # from the definition line to the first closing brace in column 0
    awk -v fn="$f" '
      $0 ~ "^void " fn "\\(" { on = 1 }
      on { print }
      on && /^}/ { on = 0; exit }
    ' "$REF/cpuLS.hpp"
  done
  cat "$HERE/ref_harness.cpp"
} | g++ -O2 -ffp-contract=off -fPIC -shared -DHAVE_UNISTD_H=1 -I"$REF" \
      -include "$HERE/ref_prelude.hpp" -x c++ - -o "$OUT/libref_cpuls.so"
echo "built $OUT/libref_cpuls.so"

# The PN correlator of the receive driver (rx_and_corr.cpp:329-360), spliced
# into oracle/pn_ref_harness.cpp in place of its marker line: from the `temp`
# vector's declaration to the closing brace of `if (corr_flag == false)`.
awk -v harness="$HERE/pn_ref_harness.cpp" '
  FNR == NR { if ($0 ~ /std::vector<std::complex<float> > temp\(num_rx_samps\);/) on = 1
              if (on) { blk = blk $0 "\n"; if ($0 ~ /if \(corr_flag == false\)/) seen = 1
                        if (seen && $0 ~ /^\t\t}$/) { on = 0; seen = 0; done = 1 } }
              next }
  /@@REFERENCE_CORRELATOR_BLOCK@@/ { if (!done) { print "#error correlator block not found"; next }
                                     printf "%s", blk; next }
  { print }
' "$REF/rx_and_corr.cpp" "$HERE/pn_ref_harness.cpp" |
  g++ -O2 -fPIC -shared -x c++ - -o "$OUT/libref_pn.so"
echo "built $OUT/libref_pn.so"
