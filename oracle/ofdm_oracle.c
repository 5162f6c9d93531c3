/*
 * ofdm_oracle.c -- CPU restatement of the reference LS + MRC path.
 *
 * TEST INFRASTRUCTURE ONLY (see ofdm_oracle.h): the checker for the HIP
 * library and the timed CPU baseline ("kind": "port") in bench.py.  Never part
 * of the product path.
 *
 * Arithmetic follows cpuLS.hpp exactly: f32 operations in the same order, the
 * naive complex divide of divideOneRow, sequential antenna sums, real-divisor
 * normalisation.  Build with -ffp-contract=off so no FMA changes the rounding
 * (the reference was built with plain g++ on x86-64, which emits no FMA).
 */
#include "ofdm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* Rotations                                                                  */
/* ------------------------------------------------------------------------ */

/* cpuLS.hpp:105-112 (matrix_readX): three memmoves on the K pilot values. */
void oracle_pilot_rotate(const oracle_cf32 *raw, int K, oracle_cf32 *X) {
    if (X != raw) memcpy(X, raw, (size_t)K * sizeof(*X));
    int nt = (K - 1) / 2;
    oracle_cf32 *tmp = (oracle_cf32 *)malloc((size_t)(nt > 0 ? nt : 1) * sizeof(*tmp));
    memmove(tmp, &X[(K + 1) / 2], (size_t)nt * sizeof(*X));
    memmove(&X[(K - 1) / 2], X, (size_t)((K + 1) / 2) * sizeof(*X));
    memmove(X, tmp, (size_t)nt * sizeof(*X));
    free(tmp);
}

/* cpuLS.hpp:135-149 (shiftOneRow with cols = K, row = 0). */
void oracle_shift_one_row(oracle_cf32 *row, int K) {
    int nt = (K + 1) / 2;
    oracle_cf32 *tmp = (oracle_cf32 *)malloc((size_t)nt * sizeof(*tmp));
    memmove(tmp, &row[(K - 1) / 2], (size_t)nt * sizeof(*row));
    memmove(&row[(K + 1) / 2], row, (size_t)((K - 1) / 2) * sizeof(*row));
    memmove(row, tmp, (size_t)nt * sizeof(*row));
    free(tmp);
}

/* ------------------------------------------------------------------------ */
/* FFT (FFTW3 forward C2C, unnormalised, sign -1: cpuLS.hpp:165-174)          */
/* Restated as the exact DFT: double-precision radix-2 DIT, rounded to f32.   */
/* ------------------------------------------------------------------------ */

#define ORACLE_MAX_LOG2 16
static double *g_tw[ORACLE_MAX_LOG2 + 1]; /* cos/sin(2*pi*k/C), k < C/2 */

static const double *twiddles(int log2c) {
    double *t = __atomic_load_n(&g_tw[log2c], __ATOMIC_ACQUIRE);
    if (t) return t;
    int C = 1 << log2c;
    int h = C / 2 > 0 ? C / 2 : 1;
    double *nt = (double *)malloc((size_t)h * 2 * sizeof(double));
    for (int k = 0; k < h; ++k) {
        double a = 2.0 * M_PI * (double)k / (double)C;
        nt[2 * k] = cos(a);
        nt[2 * k + 1] = sin(a);
    }
    double *expected = NULL;
    if (!__atomic_compare_exchange_n(&g_tw[log2c], &expected, nt, 0,
                                     __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        free(nt);
        return expected;
    }
    return nt;
}

static void fft_double(double *re, double *im, int C, int inverse) {
    int log2c = 0;
    while ((1 << log2c) < C) ++log2c;
    /* bit reversal */
    for (int i = 1, j = 0; i < C; ++i) {
        int bit = C >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
    const double *tw = twiddles(log2c);
    double sgn = inverse ? 1.0 : -1.0;
    for (int len = 2; len <= C; len <<= 1) {
        int half = len / 2, step = C / len;
        for (int i = 0; i < C; i += len) {
            for (int k = 0; k < half; ++k) {
                double wr = tw[2 * k * step], wi = sgn * tw[2 * k * step + 1];
                int a = i + k, b = i + k + half;
                double xr = re[b] * wr - im[b] * wi;
                double xi = re[b] * wi + im[b] * wr;
                re[b] = re[a] - xr; im[b] = im[a] - xi;
                re[a] += xr;        im[a] += xi;
            }
        }
    }
}

/* Any other length (the sizes FFTW takes beyond powers of two, e.g. 1536,
 * 600, odd and prime C): decimation in time by the smallest prime factor p
 * of n, X[k] = sum_{r<p} W_n^{r k} S_r[k mod n/p] with S_r the DFTs of the p
 * subsequences x[r + p i]; at prime n the direct sum.  Double precision,
 * every twiddle from cos / sin of the exact angle 2 pi ((r k) mod n) / n. */
static void dft_any(const double *xr, const double *xi, size_t stride, int n, double *yr, double *yi,
                    double sgn) {
    if (n == 1) { yr[0] = xr[0]; yi[0] = xi[0]; return; }
    int p = 2;
    while (p * p <= n && n % p) ++p;
    if (n % p) p = n;
    const int m = n / p;
    double *sr = (double *)malloc((size_t)n * sizeof(double));
    double *si = (double *)malloc((size_t)n * sizeof(double));
    if (p == n) { /* prime: the subsequences are single samples */
        for (int r = 0; r < n; ++r) { sr[r] = xr[r * stride]; si[r] = xi[r * stride]; }
    } else {
        for (int r = 0; r < p; ++r)
            dft_any(xr + r * stride, xi + r * stride, stride * p, m, sr + (size_t)r * m, si + (size_t)r * m, sgn);
    }
    for (int k = 0; k < n; ++k) {
        double ar = 0.0, ai = 0.0;
        for (int r = 0; r < p; ++r) {
            const double a = 2.0 * M_PI * (double)(((long long)r * k) % n) / (double)n;
            const double wr = cos(a), wi = sgn * sin(a);
            const double vr = sr[(size_t)r * m + k % m], vi = si[(size_t)r * m + k % m];
            ar += vr * wr - vi * wi;
            ai += vr * wi + vi * wr;
        }
        yr[k] = ar;
        yi[k] = ai;
    }
    free(sr);
    free(si);
}

void oracle_fft_row(oracle_cf32 *row, int C, int inverse) {
    if (C < 1) return;
    if (C & (C - 1)) { /* not a power of two */
        double *xr = (double *)malloc((size_t)C * 4 * sizeof(double));
        double *xi = xr + C, *yr = xr + 2 * (size_t)C, *yi = xr + 3 * (size_t)C;
        for (int i = 0; i < C; ++i) { xr[i] = row[i].re; xi[i] = row[i].im; }
        dft_any(xr, xi, 1, C, yr, yi, inverse ? 1.0 : -1.0);
        for (int i = 0; i < C; ++i) { row[i].re = (float)yr[i]; row[i].im = (float)yi[i]; }
        free(xr);
        return;
    }
    double stack_re[4096], stack_im[4096];
    double *re = stack_re, *im = stack_im;
    if (C > 4096) {
        re = (double *)malloc((size_t)C * sizeof(double));
        im = (double *)malloc((size_t)C * sizeof(double));
    }
    for (int i = 0; i < C; ++i) { re[i] = row[i].re; im[i] = row[i].im; }
    fft_double(re, im, C, inverse);
    for (int i = 0; i < C; ++i) { row[i].re = (float)re[i]; row[i].im = (float)im[i]; }
    if (C > 4096) { free(re); free(im); }
}

/* Single-precision variant, for the timed CPU baseline only (bench.py
 * cpu_baseline): the reference calls FFTW's single-precision fftwf
 * (cpuLS.hpp:157-159, 170-172), so the baseline should not pay for a float64
 * transform.  Same radix-2 DIT structure, f32 arithmetic, f32 twiddle table
 * (the reference re-plans per row; here the table is reused).
 * Results agree with the float64 form to f32 rounding of the FFT (~1e-6
 * relative), which is NOT the parity path: parity uses oracle_fft_row. */
static float *g_tw32[ORACLE_MAX_LOG2 + 1];

static const float *twiddles32(int log2c) {
    float *t = __atomic_load_n(&g_tw32[log2c], __ATOMIC_ACQUIRE);
    if (t) return t;
    int C = 1 << log2c;
    int h = C / 2 > 0 ? C / 2 : 1;
    const double *td = twiddles(log2c);
    float *nt = (float *)malloc((size_t)h * 2 * sizeof(float));
    for (int k = 0; k < 2 * h; ++k) nt[k] = (float)td[k];
    float *expected = NULL;
    if (!__atomic_compare_exchange_n(&g_tw32[log2c], &expected, nt, 0,
                                     __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        free(nt);
        return expected;
    }
    return nt;
}

void oracle_fft_row_f32(oracle_cf32 *row, int C) {
    float re[4096], im[4096];
    if (C > 4096 || (C & (C - 1))) { oracle_fft_row(row, C, 0); return; }
    int log2c = 0;
    while ((1 << log2c) < C) ++log2c;
    for (int i = 0; i < C; ++i) { re[i] = row[i].re; im[i] = row[i].im; }
    for (int i = 1, j = 0; i < C; ++i) {
        int bit = C >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            float t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
    const float *tw = twiddles32(log2c);
    for (int len = 2; len <= C; len <<= 1) {
        int half = len / 2, step = C / len;
        for (int i = 0; i < C; i += len) {
            for (int k = 0; k < half; ++k) {
                float wr = tw[2 * k * step], wi = -tw[2 * k * step + 1];
                int a = i + k, b = i + k + half;
                float xr = re[b] * wr - im[b] * wi;
                float xi = re[b] * wi + im[b] * wr;
                re[b] = re[a] - xr; im[b] = im[a] - xi;
                re[a] += xr;        im[a] += xi;
            }
        }
    }
    for (int i = 0; i < C; ++i) { row[i].re = re[i]; row[i].im = im[i]; }
}

/* ------------------------------------------------------------------------ */
/* LS channel estimate (firstVector, cpuLS.hpp:290-311)                      */
/* ------------------------------------------------------------------------ */
void oracle_ls(const oracle_cf32 *Yfft, const oracle_cf32 *X, int R, int C,
               oracle_cf32 *Hconj, float *Hsqrd) {
    int K = C - 1;
    for (int r = 0; r < R; ++r) {
        /* memcpy(&Hconj[row*(cols-1)], &Y[row*cols+1], ...)  (290-292) */
        const oracle_cf32 *y = &Yfft[(size_t)r * C + 1];
        oracle_cf32 *h = &Hconj[(size_t)r * K];
        /* divideOneRow (cpuLS.hpp:233-244): naive formula */
        for (int j = 0; j < K; ++j) {
            float fxa = y[j].re, fxb = y[j].im;
            float fya = X[j].re, fyb = X[j].im;
            h[j].re = (fxa * fya + fxb * fyb) / (fya * fya + fyb * fyb);
            h[j].im = (fxb * fya - fxa * fyb) / (fya * fya + fyb * fyb);
        }
    }
    /* conjugate (303-307): imag = -1 * imag */
    for (size_t i = 0; i < (size_t)R * K; ++i) Hconj[i].im = -1 * Hconj[i].im;
    /* findDistSqrd (cpuLS.hpp:211-228), sequential over rows */
    for (int j = 0; j < K; ++j)
        Hsqrd[j] = (Hconj[j].re * Hconj[j].re) + (Hconj[j].im * Hconj[j].im);
    for (int r = 1; r < R; ++r)
        for (int j = 0; j < K; ++j) {
            const oracle_cf32 h = Hconj[(size_t)r * K + j];
            Hsqrd[j] = Hsqrd[j] + (h.re * h.re) + (h.im * h.im);
        }
}

/* ------------------------------------------------------------------------ */
/* MRC (doOneSymbol, cpuLS.hpp:354-368)                                        */
/* ------------------------------------------------------------------------ */
void oracle_mrc_numerator(const oracle_cf32 *Yfft, const oracle_cf32 *Hconj,
                          int R, int C, oracle_cf32 *num) {
    int K = C - 1;
    /* matrixMultThenSum (cpuLS.hpp:187-208) on Ytemp = Y without bin 0 */
    for (int i = 0; i < R; ++i) {
        const oracle_cf32 *y = &Yfft[(size_t)i * C + 1];
        const oracle_cf32 *h = &Hconj[(size_t)i * K];
        for (int j = 0; j < K; ++j) {
            float Yreal = y[j].re, Yimag = y[j].im;
            float Hreal = h[j].re, Himag = h[j].im;
            if (i == 0) { num[j].re = 0; num[j].im = 0; }
            num[j].re = num[j].re + (Yreal * Hreal - Yimag * Himag);
            num[j].im = num[j].im + (Yreal * Himag + Yimag * Hreal);
        }
    }
}

void oracle_mrc(const oracle_cf32 *Yfft, const oracle_cf32 *Hconj,
                const float *Hsqrd, int R, int C, oracle_cf32 *out) {
    int K = C - 1;
    oracle_mrc_numerator(Yfft, Hconj, R, C, out);
    /* normalise (364-367): two real divides */
    for (int j = 0; j < K; ++j) {
        out[j].re = out[j].re / Hsqrd[j];
        out[j].im = out[j].im / Hsqrd[j];
    }
    oracle_shift_one_row(out, K); /* (368) */
}

/* ------------------------------------------------------------------------ */
/* Frames                                                                       */
/* ------------------------------------------------------------------------ */
static void load_symbol(const oracle_cf32 *sym, int R, int C, int prefix,
                        oracle_cf32 *Y, int fft32) {
    /* ShMemSymBuff.hpp:309-322: drop the prefix of each row */
    for (int r = 0; r < R; ++r)
        memcpy(&Y[(size_t)r * C], &sym[(size_t)r * (C + prefix) + prefix],
               (size_t)C * sizeof(*Y));
    /* fftOneRow per antenna row (cpuLS.hpp:278-281, 342-345) */
    for (int r = 0; r < R; ++r) {
        if (fft32 == 2)
            oracle_fft_row_fast(&Y[(size_t)r * C], C);
        else if (fft32)
            oracle_fft_row_f32(&Y[(size_t)r * C], C);
        else
            oracle_fft_row(&Y[(size_t)r * C], C, 0);
    }
}

static void frame_demod_ex(const oracle_cf32 *iq, int S, int R, int C, int prefix,
                           const oracle_cf32 *X, oracle_cf32 *out,
                           oracle_cf32 *Hconj, float *Hsqrd, int fft32);

void oracle_frame_demod(const oracle_cf32 *iq, int S, int R, int C, int prefix,
                        const oracle_cf32 *X, oracle_cf32 *out,
                        oracle_cf32 *Hconj, float *Hsqrd) {
    frame_demod_ex(iq, S, R, C, prefix, X, out, Hconj, Hsqrd, 0);
}

static void frame_demod_ex(const oracle_cf32 *iq, int S, int R, int C, int prefix,
                           const oracle_cf32 *X, oracle_cf32 *out,
                           oracle_cf32 *Hconj, float *Hsqrd, int fft32) {
    int K = C - 1;
    size_t sym_elems = (size_t)R * (C + prefix);
    oracle_cf32 *Y = (oracle_cf32 *)malloc((size_t)R * C * sizeof(*Y));
    oracle_cf32 *H = Hconj ? Hconj : (oracle_cf32 *)malloc((size_t)R * K * sizeof(*H));
    float *P = Hsqrd ? Hsqrd : (float *)malloc((size_t)K * sizeof(*P));
    load_symbol(iq, R, C, prefix, Y, fft32);
    oracle_ls(Y, X, R, C, H, P);
    for (int s = 1; s < S; ++s) {
        load_symbol(iq + (size_t)s * sym_elems, R, C, prefix, Y, fft32);
        oracle_mrc(Y, H, P, R, C, out + (size_t)(s - 1) * K);
    }
    free(Y);
    if (!Hconj) free(H);
    if (!Hsqrd) free(P);
}

void oracle_frames_demod(const oracle_cf32 *iq, long long nframes, int S, int R,
                         int C, int prefix, const oracle_cf32 *X,
                         oracle_cf32 *out, int nthreads) {
    size_t frame_elems = (size_t)S * R * (C + prefix);
    size_t out_elems = (size_t)(S - 1) * (C - 1);
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (long long f = 0; f < nframes; ++f)
        oracle_frame_demod(iq + f * frame_elems, S, R, C, prefix, X,
                           out + f * out_elems, NULL, NULL);
    (void)nthreads;
}

void oracle_frames_demod_fft32(const oracle_cf32 *iq, long long nframes, int S, int R,
                               int C, int prefix, const oracle_cf32 *X,
                               oracle_cf32 *out, int nthreads) {
    size_t frame_elems = (size_t)S * R * (C + prefix);
    size_t out_elems = (size_t)(S - 1) * (C - 1);
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (long long f = 0; f < nframes; ++f)
        frame_demod_ex(iq + f * frame_elems, S, R, C, prefix, X,
                       out + f * out_elems, NULL, NULL, 1);
    (void)nthreads;
}

void oracle_frames_demod_fftfast(const oracle_cf32 *iq, long long nframes, int S, int R,
                                 int C, int prefix, const oracle_cf32 *X,
                                 oracle_cf32 *out, int nthreads) {
    size_t frame_elems = (size_t)S * R * (C + prefix);
    size_t out_elems = (size_t)(S - 1) * (C - 1);
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (long long f = 0; f < nframes; ++f)
        frame_demod_ex(iq + f * frame_elems, S, R, C, prefix, X,
                       out + f * out_elems, NULL, NULL, 2);
    (void)nthreads;
}

void oracle_frames_demod_freq(const oracle_cf32 *yf, long long nframes, int S,
                              int R, int C, const oracle_cf32 *X,
                              oracle_cf32 *out, int nthreads) {
    int K = C - 1;
    size_t frame_elems = (size_t)S * R * C;
    size_t out_elems = (size_t)(S - 1) * K;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (long long f = 0; f < nframes; ++f) {
        oracle_cf32 *H = (oracle_cf32 *)malloc((size_t)R * K * sizeof(*H));
        float *P = (float *)malloc((size_t)K * sizeof(*P));
        const oracle_cf32 *fr = yf + f * frame_elems;
        oracle_ls(fr, X, R, C, H, P);
        for (int s = 1; s < S; ++s)
            oracle_mrc(fr + (size_t)s * R * C, H, P, R, C,
                       out + f * out_elems + (size_t)(s - 1) * K);
        free(H);
        free(P);
    }
    (void)nthreads;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
