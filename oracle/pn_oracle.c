/*
 * pn_oracle.c -- CPU restatement of the reference's PN frame-sync correlator
 * and frame extraction (rx_and_corr.cpp).
 *
 * TEST INFRASTRUCTURE ONLY (see ofdm_oracle.h): the checker for the HIP
 * correlator (ofdm_pn_correlate / ofdm_pn_extract).  Never part of the
 * product path.
 *
 * The reference loop lives inside UHD_SAFE_MAIN next to the radio streaming
 * calls (uhd, boost), so it cannot be compiled here; this restates it line
 * for line.  Arithmetic: std::complex<float> product (ac - bd, ad + bc) and
 * sum in f32, sequential j, no FMA (-ffp-contract=off, as plain g++ on
 * x86-64 emits none); std::abs(complex<float>) is cabsf (glibc hypotf);
 * division by (float)pn_buff.size().
 */
#include <complex.h>
#include <math.h>
#include <string.h>

#include "ofdm_oracle.h"

/* rx_and_corr.cpp:341-353: one lag */
static float corr_mag(const oracle_cf32 *x, const oracle_cf32 *pn, int L) {
    float tr = 0.f, ti = 0.f;
    for (int j = 0; j < L; j++) {
        const float a = pn[j].re, b = pn[j].im, c = x[j].re, d = x[j].im;
        const float pr = a * c - b * d;
        const float pi = a * d + b * c;
        tr = tr + pr;
        ti = ti + pi;
    }
    return cabsf(CMPLXF(tr, ti)) / (float)L;
}

/* rx_and_corr.cpp:332-360 (the corr_flag == false branch) */
void oracle_pn_correlate(const oracle_cf32 *buf, int R, long long N, const oracle_cf32 *pn,
                         int L, float thres, long long *pos, float *mag) {
    const long long nl = N - L + 1;
    *pos = -1;
    if (nl <= 0 || L <= 0) return;
    for (int ch = 0; ch < R; ch++) {
        const oracle_cf32 *x = buf + (long long)ch * N;
        for (long long i = 0; i < nl; i++) {
            const float v = corr_mag(x + i, pn, L);
            if (mag) mag[(long long)ch * nl + i] = v;
            if (v >= thres && *pos < 0) {
                *pos = (long long)ch * nl + i;
                if (!mag) return; /* length = i; corr_flag = true; break (both loops) */
            }
        }
    }
}

/* rx_and_corr.cpp:370-392 (copy_buff from buff1 after the PN, then the first
 * `length` samples of buff2) and copy_to_shared_mem (64-87: per symbol, per
 * channel, FFT_size samples after the cyclic prefix). */
void oracle_pn_extract(const oracle_cf32 *buf1, const oracle_cf32 *buf2, int R, long long N,
                       int L, long long lag, int C, int cp, int nsym, oracle_cf32 *sym) {
    for (int ch = 0; ch < R; ch++) {
        const oracle_cf32 *b1 = buf1 + (long long)ch * N, *b2 = buf2 + (long long)ch * N;
        for (int s = 0; s < nsym; s++)
            for (int k = 0; k < C; k++) {
                const long long q = (long long)s * (C + cp) + cp + k; /* index into copy_buff[ch] */
                const long long head = N - lag - L;                 /* samples taken from buff1 */
                oracle_cf32 v = q < head ? b1[lag + L + q] : b2[q - head];
                sym[((long long)s * R + ch) * C + k] = v;
            }
    }
}
