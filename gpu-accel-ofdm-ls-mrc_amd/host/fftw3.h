// fftw3.h -- the single-precision FFTW calls the reference's CPU receiver
// makes, served by the MI355X library.
//
// The reference's cpuLS.hpp (cpuLS.hpp:31) and cpuLS_main.cpp (cpuLS_main.cpp:28)
// include <fftw3.h>; the receiver transforms one antenna row at a time with
// fftwf_plan_dft_1d + fftwf_execute + fftwf_destroy_plan (fftOneRow /
// ifftOneRow, cpuLS.hpp:152-174).  This header declares exactly that subset so
// the drivers build unchanged on a machine without FFTW: a plan records its
// size, arrays and sign, and executing it runs ofdm_fft_rows (unnormalised
// C2C, the FFTW sign convention: FFTW_FORWARD = e^{-2 pi i jk/n}) on the GPU
// through the host staging engine.  Sizes are the library's: any n in
// [2, 8192] (n = 1 is the identity); any other n aborts with a message (no CPU
// fallback).
// Planning never touches the arrays (FFTW_MEASURE's clobbering, which the
// reference works around at cpuLS.hpp:262, does not happen).
//
// Everything here is `inline` in the C++ sense, so a translation unit that
// also links the real libfftw3f sees no duplicate symbols; do not put this
// directory on the include path where the real <fftw3.h> is wanted.
#ifndef OFDM_FFTW3_SUBSET_H_
#define OFDM_FFTW3_SUBSET_H_

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ofdm_engine.hpp"

#define FFTW_FORWARD (-1)
#define FFTW_BACKWARD (+1)
#define FFTW_MEASURE (0U)
#define FFTW_DESTROY_INPUT (1U << 0)
#define FFTW_UNALIGNED (1U << 1)
#define FFTW_EXHAUSTIVE (1U << 3)
#define FFTW_PRESERVE_INPUT (1U << 4)
#define FFTW_PATIENT (1U << 5)
#define FFTW_ESTIMATE (1U << 6)

typedef float fftwf_complex[2];

struct ofdm_fftwf_plan_s {
    int n;
    fftwf_complex *in, *out;
    int sign;
};
typedef ofdm_fftwf_plan_s *fftwf_plan;

inline fftwf_plan fftwf_plan_dft_1d(int n, fftwf_complex *in, fftwf_complex *out, int sign,
                                    unsigned /*flags*/) {
    if (n < 1 || n > 8192) {
        std::fprintf(stderr, "fftwf_plan_dft_1d: n=%d unsupported (1 <= n <= 8192)\n", n);
        std::abort();
    }
    return new ofdm_fftwf_plan_s{n, in, out, sign};
}

inline void fftwf_execute(const fftwf_plan p) {
    if (p->out != p->in) std::memcpy(p->out, p->in, sizeof(fftwf_complex) * (size_t)p->n);
    if (p->n == 1) return;  // the DFT of one sample is itself
    ofdm::HostEngine::get().fft_rows(p->out, 1, p->n, p->sign == FFTW_BACKWARD ? 1 : 0);
}

inline void fftwf_destroy_plan(fftwf_plan p) { delete p; }

inline void *fftwf_malloc(size_t n) { return std::malloc(n); }
inline void fftwf_free(void *p) { std::free(p); }
inline void fftwf_cleanup() {}

#endif  // OFDM_FFTW3_SUBSET_H_
