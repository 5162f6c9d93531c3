/*
 * zf_oracle.c -- CPU restatement of the reference's zero-forcing precoder
 * (cpuLS.hpp:401-466: rotCube, createZeroForcingMatrix,
 * multiplyWithChannelInv).
 *
 * TEST INFRASTRUCTURE ONLY (see ofdm_oracle.h): the checker for the HIP
 * ZF kernels.  Never part of the product path.
 *
 * The reference calls CBLAS (cgemm, cgemv) and LAPACK (cgetrf, cgetri); none
 * is installed here, so their published algorithms are
 * restated in single-precision complex: straightforward cgemm / cgemv sums,
 * unblocked LU with partial pivoting (LAPACK cgetf2: pivot = first max of
 * |re| + |im|, icamax), and cgetri's inverse (invert U, solve inv(A) L =
 * inv(U), undo the column interchanges); complex reciprocals by Smith's
 * algorithm, as gfortran compiles LAPACK's ONE / A(J,J).
 */
#include <complex.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ofdm_oracle.h"

typedef float _Complex cf;

static inline cf ld(const oracle_cf32 *p) { return CMPLXF(p->re, p->im); }
static inline void st(oracle_cf32 *p, cf v) {
    p->re = crealf(v);
    p->im = cimagf(v);
}
static inline float cabs1(cf v) { return fabsf(crealf(v)) + fabsf(cimagf(v)); }

/* 1 / a by Smith's algorithm: LAPACK's ONE / A(J,J) (cgetf2, ctrti2) under
 * gfortran's complex-division rules (-fcx-fortran-rules: Smith, no scaling),
 * rather than C's __divsc3. */
static inline cf crcp(cf a) {
    const float c = crealf(a), d = cimagf(a);
    if (fabsf(c) >= fabsf(d)) {
        const float r = d / c, den = c + d * r;
        return CMPLXF(1.0f / den, -r / den);
    }
    const float r = c / d, den = c * r + d;
    return CMPLXF(r / den, -1.0f / den);
}

/* cgetrf (unblocked cgetf2) on an n x n column-major matrix a (lda = n) */
static int lu(cf *a, int n, int *ipiv) {
    int info = 0;
    for (int j = 0; j < n; j++) {
        int p = j;
        for (int i = j + 1; i < n; i++)
            if (cabs1(a[j * n + i]) > cabs1(a[j * n + p])) p = i;
        ipiv[j] = p;
        if (a[j * n + p] != 0) {
            if (p != j)
                for (int c = 0; c < n; c++) {
                    cf t = a[c * n + j];
                    a[c * n + j] = a[c * n + p];
                    a[c * n + p] = t;
                }
            const cf r = crcp(a[j * n + j]);
            for (int i = j + 1; i < n; i++) a[j * n + i] *= r;
        } else if (!info) {
            info = j + 1;
        }
        for (int c = j + 1; c < n; c++)
            for (int i = j + 1; i < n; i++) a[c * n + i] -= a[j * n + i] * a[c * n + j];
    }
    return info;
}

/* cgetri: inverse from the LU factors (column-major, in place) */
static void lu_inverse(cf *a, int n, const int *ipiv) {
    /* ctrtri: invert the upper triangle U in place (unblocked ctrti2, non-unit) */
    for (int j = 0; j < n; j++) {
        a[j * n + j] = crcp(a[j * n + j]);
        const cf ajj = -a[j * n + j];
        /* x = triu(inv(U))[0..j-1, 0..j-1] * a[0..j-1, j]  (ctrmv, upper, no-trans) */
        for (int c = 0; c < j; c++) {
            const cf t = a[j * n + c];
            for (int i = 0; i < c; i++) a[j * n + i] += t * a[c * n + i];
            a[j * n + c] = t * a[c * n + c];
        }
        for (int i = 0; i < j; i++) a[j * n + i] *= ajj;
    }
    /* solve inv(A) * L = inv(U) for inv(A), columns right to left */
    cf *work = (cf *)malloc((size_t)n * sizeof(cf));
    for (int j = n - 1; j >= 0; j--) {
        for (int i = j + 1; i < n; i++) {
            work[i] = a[j * n + i];
            a[j * n + i] = 0;
        }
        for (int c = j + 1; c < n; c++)
            for (int i = 0; i < n; i++) a[j * n + i] -= a[c * n + i] * work[c];
    }
    free(work);
    /* undo the row interchanges as column interchanges, last first */
    for (int j = n - 2; j >= 0; j--) {
        const int p = ipiv[j];
        if (p != j)
            for (int i = 0; i < n; i++) {
                cf t = a[j * n + i];
                a[j * n + i] = a[p * n + i];
                a[p * n + i] = t;
            }
    }
}

void oracle_zf_precoder(const oracle_cf32 *Hin, int users, int rows, int K, oracle_cf32 *W) {
    const int U = users, R = rows;
    cf *A = (cf *)malloc((size_t)U * R * sizeof(cf)); /* X[col] after rotCube: A[r*U + u] */
    cf *G = (cf *)malloc((size_t)U * U * sizeof(cf));
    int *ipiv = (int *)malloc((size_t)U * sizeof(int));
    for (int k = 0; k < K; k++) {
        for (int r = 0; r < R; r++)
            for (int u = 0; u < U; u++) A[r * U + u] = ld(&Hin[((long long)u * R + r) * K + k]);
        /* cgemm(ColMajor, NoTrans, ConjTrans, U, U, R): G[a][b] = sum_r A(a,r) conj(A(b,r)) */
        for (int b = 0; b < U; b++)
            for (int a = 0; a < U; a++) {
                cf s = 0;
                for (int r = 0; r < R; r++) s += A[r * U + a] * conjf(A[r * U + b]);
                G[b * U + a] = s;
            }
        lu(G, U, ipiv);
        lu_inverse(G, U, ipiv);
        /* cgemm(ColMajor, ConjTrans, NoTrans, R, U, U): W(r,u) = sum_a conj(A(a,r)) Ginv(a,u) */
        for (int u = 0; u < U; u++)
            for (int r = 0; r < R; r++) {
                cf s = 0;
                for (int a = 0; a < U; a++) s += conjf(A[r * U + a]) * G[u * U + a];
                st(&W[(long long)k * R * U + (long long)u * R + r], s);
            }
    }
    free(A);
    free(G);
    free(ipiv);
}

void oracle_zf_apply(const oracle_cf32 *W, const oracle_cf32 *X, int users, int rows, int K,
                     int nsym, oracle_cf32 *Y) {
    for (int s = 0; s < nsym; s++)
        for (int k = 0; k < K; k++)
            for (int r = 0; r < rows; r++) {
                cf acc = 0;
                for (int u = 0; u < users; u++)
                    acc += ld(&W[(long long)k * rows * users + (long long)u * rows + r]) *
                           ld(&X[((long long)s * users + u) * K + k]);
                st(&Y[((long long)s * rows + r) * K + k], acc);
            }
}

void oracle_zf_detect(const oracle_cf32 *W, const oracle_cf32 *Y, int users, int rows, int K,
                      int nsym, oracle_cf32 *X) {
    for (int s = 0; s < nsym; s++)
        for (int k = 0; k < K; k++)
            for (int u = 0; u < users; u++) {
                cf acc = 0;
                for (int r = 0; r < rows; r++)
                    acc += conjf(ld(&W[(long long)k * rows * users + (long long)u * rows + r])) *
                           ld(&Y[((long long)s * rows + r) * K + k]);
                st(&X[((long long)s * users + u) * K + k], acc);
            }
}
