/* fft_fast.c -- TEST INFRASTRUCTURE ONLY (bench.py's timed CPU baseline).
 *
 * A single-precision complex FFT for power-of-two sizes written so that the
 * compiler vectorises it (AVX2 code generation in fft_row_avx2 only, entered
 * behind a runtime CPU check; -ffp-contract=off, so no FMA contraction):
 * split real / imaginary arrays, a precomputed bit-reversal table, and per
 * stage a contiguous twiddle table (stage of half-length h: w[h + k] =
 * exp(-2 pi i k / 2h), k < h), so the butterfly loop over k reads every
 * operand with unit stride.  It stands in for the reference's fftwf plans
 * (cpuLS.hpp:278-281 fftOneRow), whose SIMD codelets are not available here;
 * it is NOT the parity oracle (ofdm_oracle.c's FFTs are): results agree with
 * them to float rounding, tests/test_oracle.py checks that.  Sizes that are
 * not powers of two, or above 8192, fall back to oracle_fft_row_f32. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ofdm_oracle.h"

typedef struct {
    int C;
    int *rev;       /* [C] bit-reversed index */
    float *wr, *wi; /* [C] per-stage twiddles at offset h */
} plan_t;

static plan_t *volatile g_plan[14];

static const plan_t *plan_for(int log2c) {
    plan_t *p = g_plan[log2c];
    if (p) return p;
    const int C = 1 << log2c;
    plan_t *np = (plan_t *)malloc(sizeof(plan_t));
    np->C = C;
    np->rev = (int *)malloc(sizeof(int) * C);
    np->wr = (float *)malloc(sizeof(float) * C);
    np->wi = (float *)malloc(sizeof(float) * C);
    for (int i = 0; i < C; ++i) {
        int r = 0;
        for (int b = 0; b < log2c; ++b) r |= ((i >> b) & 1) << (log2c - 1 - b);
        np->rev[i] = r;
    }
    np->wr[0] = 1.f;
    np->wi[0] = 0.f;
    for (int h = 1; h < C; h <<= 1)
        for (int k = 0; k < h; ++k) {
            const double a = -M_PI * (double)k / (double)h;
            np->wr[h + k] = (float)cos(a);
            np->wi[h + k] = (float)sin(a);
        }
    plan_t *expected = NULL;
    if (!__atomic_compare_exchange_n(&g_plan[log2c], &expected, np, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        free(np->rev); free(np->wr); free(np->wi); free(np);
        return expected;
    }
    return np;
}

/* the vectorised body: AVX2 code generation for this function only, entered
 * only on a CPU that has AVX2 (oracle_fft_row_fast below) */
__attribute__((target("avx2"))) static void fft_row_avx2(oracle_cf32 *row, int C) {
    int log2c = 0;
    while ((1 << log2c) < C) ++log2c;
    const plan_t *p = plan_for(log2c);
    float re[8192] __attribute__((aligned(64))), im[8192] __attribute__((aligned(64)));
    for (int i = 0; i < C; ++i) {
        const oracle_cf32 v = row[p->rev[i]];
        re[i] = v.re;
        im[i] = v.im;
    }
    /* stages 1 and 2 as one radix-4 step (twiddles 1 and -i) */
    for (int i = 0; i < C; i += 4) {
        const float a0r = re[i] + re[i + 1], a0i = im[i] + im[i + 1];
        const float a1r = re[i] - re[i + 1], a1i = im[i] - im[i + 1];
        const float b0r = re[i + 2] + re[i + 3], b0i = im[i + 2] + im[i + 3];
        const float b1r = re[i + 2] - re[i + 3], b1i = im[i + 2] - im[i + 3];
        re[i] = a0r + b0r;     im[i] = a0i + b0i;
        re[i + 2] = a0r - b0r; im[i + 2] = a0i - b0i;
        re[i + 1] = a1r + b1i; im[i + 1] = a1i - b1r;  /* a1 + (-i) b1 */
        re[i + 3] = a1r - b1i; im[i + 3] = a1i + b1r;
    }
    for (int h = 4; h < C; h <<= 1) {
        const float *restrict wr = p->wr + h, *restrict wi = p->wi + h;
        for (int i = 0; i < C; i += 2 * h) {
            float *restrict ar = re + i, *restrict ai = im + i;
            float *restrict br = re + i + h, *restrict bi = im + i + h;
            for (int k = 0; k < h; ++k) {
                const float xr = br[k] * wr[k] - bi[k] * wi[k];
                const float xi = br[k] * wi[k] + bi[k] * wr[k];
                br[k] = ar[k] - xr;
                bi[k] = ai[k] - xi;
                ar[k] = ar[k] + xr;
                ai[k] = ai[k] + xi;
            }
        }
    }
    for (int i = 0; i < C; ++i) {
        row[i].re = re[i];
        row[i].im = im[i];
    }
}

void oracle_fft_row_fast(oracle_cf32 *row, int C) {
    if (C < 4 || C > 8192 || (C & (C - 1)) || !__builtin_cpu_supports("avx2")) {
        oracle_fft_row_f32(row, C);  /* the same butterflies in the same order: identical bits */
        return;
    }
    fft_row_avx2(row, C);
}
