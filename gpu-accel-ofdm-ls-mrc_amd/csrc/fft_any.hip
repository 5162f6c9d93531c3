// fft_any.hip -- batched row FFT of ANY length C in [2, 8192] (mixed radix,
// Stockham autosort in LDS), for the sizes the power-of-two kernels
// (k_fft_rows, the fused receivers) do not cover: 1536 (LTE 15 MHz), 600,
// 1200, odd and prime lengths, 8192.  The reference transforms whatever
// `dimension` it is built with (ShMemSymBuff.hpp:47) through FFTW
// (fftOneRow, cpuLS.hpp:165-174) or cuFFT (gpuLS.cu:94-97, 377-381), both
// size-generic; this kernel is what makes the staged path of the library
// size-generic too.  Unnormalised, forward sign -1 (inverse +1, then `scale`).
//
// Algorithm (C = p_1 p_2 ... p_n, one Stockham stage per factor):
//   after the stages with radices whose product is L', the row holds
//   y[m][k] = DFT_{L'} of the subsequence x[m + n M'] (M' = C / L'), stored
//   at m L' + k.  A stage of radix p (L = L' p, cp = C / p) forms, for each
//   butterfly b = m L' + k1 (b < cp):
//     a_t = W_L^{t k1} y[b + t cp],  t < p
//     y'[m L + k1 + L' k2] = sum_t W_p^{t k2} a_t,  k2 < p
//   which ends in natural order (L = C).  Radices 8, 4, 2 run as in-register
//   FFTs with compile-time twiddles (common.hpp fft_reg), 3, 5, 7 as direct
//   DFTs with their p - 1 roots held in registers; any other prime factor
//   runs one output per thread, sum_t W_L^{(t k) mod L} y[b + t cp] over the
//   p inputs, accumulated in double (products of two floats are exact in
//   double) and rounded once.
//
// Layout: one workgroup (256 threads) owns G rows at a time (G C <= 4096 in
// the small variant, 64 KiB of LDS with the table; one row of up to 8192 in
// the big variant, 128 KiB) and walks the row groups of the batch
// persistently.  W_C^e, e < C, is computed once per workgroup into LDS in
// double precision (sincospi) and rounded to float.  Every stage reads all
// its inputs into registers, synchronises, and writes its outputs over them
// (in place, one buffer).  The data is HBM-bound in principle (one read and
// one write of the row); the stages are LDS and VALU work.
#include "common.hpp"
#include "launch.hpp"

namespace ofdm {
namespace fany {

constexpr int NT = 256;
constexpr int MAX_STAGES = 16;

struct Plan {
    int C, G, ns;
    int p[MAX_STAGES];
};

template <bool INV>
__device__ __forceinline__ float2 twv(const float2 *tw, int e) {
    const float2 w = tw[e];
    return INV ? float2{w.x, -w.y} : w;
}

// radices 2, 4, 8: in-register FFT (compile-time twiddles);
// 3, 5, 7: direct DFT with the roots r[j] = W_p^j held in registers
template <int P, bool INV>
__device__ __forceinline__ void dft_small(float2 (&a)[P], const float2 (&r)[P]) {
    if constexpr (P == 2 || P == 4 || P == 8) {
        fft_reg<P, INV>(a);
    } else {
        float2 y[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            float2 s = a[0];
#pragma unroll
            for (int t = 1; t < P; ++t) {
                const float2 w = r[(t * k) % P];
                s = float2{s.x + (a[t].x * w.x - a[t].y * w.y), s.y + (a[t].x * w.y + a[t].y * w.x)};
            }
            y[k] = s;
        }
#pragma unroll
        for (int k = 0; k < P; ++k) a[k] = y[k];
    }
}

// one stage of radix P over G rows of x (in place): read all, sync, write all
template <int P, int MAXE, bool INV>
__device__ __forceinline__ void stage_small(float2 *x, const float2 *tw, unsigned C, unsigned G, unsigned Lp) {
    constexpr int MAXB = (MAXE + P - 1) / P;
    const unsigned cp = C / P, nb = G * cp, M = cp / Lp;
    float2 r[P];
#pragma unroll
    for (int j = 0; j < P; ++j) r[j] = (P == 3 || P == 5 || P == 7) ? twv<INV>(tw, j * cp) : float2{1.f, 0.f};
    float2 v[MAXB][P];
    unsigned ob[MAXB];
#pragma unroll
    for (int q = 0; q < MAXB; ++q) {
        const unsigned bb = threadIdx.x + q * NT;
        ob[q] = ~0u;
        if (bb < nb) {
            const unsigned g = bb / cp, b = bb - g * cp, m = b / Lp, k1 = b - m * Lp;
            const float2 *src = x + g * C + b;
#pragma unroll
            for (int t = 0; t < P; ++t) {
                float2 a = src[t * cp];
                if (t > 0 && k1 != 0) a = cmul(a, twv<INV>(tw, t * k1 * M));
                v[q][t] = a;
            }
            ob[q] = g * C + m * Lp * P + k1;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < MAXB; ++q) {
        if (ob[q] != ~0u) {
            dft_small<P, INV>(v[q], r);
#pragma unroll
            for (int k2 = 0; k2 < P; ++k2) x[ob[q] + k2 * Lp] = v[q][k2];
        }
    }
    __syncthreads();
}

// one stage of any radix p: one output per thread slot, double accumulation
template <int MAXE, bool INV>
__device__ __forceinline__ void stage_any(float2 *x, const float2 *tw, unsigned C, unsigned G, unsigned Lp,
                                          unsigned p) {
    const unsigned L = Lp * p, cp = C / p, M = C / L, n = G * C;
    float2 res[MAXE];
#pragma unroll
    for (int q = 0; q < MAXE; ++q) {
        const unsigned o = threadIdx.x + q * NT;
        if (o < n) {
            const unsigned g = o / C, pos = o - g * C, m = pos / L, k = pos - m * L, k1 = k % Lp;
            const float2 *src = x + g * C + m * Lp + k1;
            double ar = 0.0, ai = 0.0;
            unsigned e = 0;
            for (unsigned t = 0; t < p; ++t) {
                const float2 a = src[t * cp];
                const float2 w = twv<INV>(tw, e * M);
                ar += (double)a.x * (double)w.x - (double)a.y * (double)w.y;
                ai += (double)a.x * (double)w.y + (double)a.y * (double)w.x;
                e += k;
                if (e >= L) e -= L;
            }
            res[q] = float2{(float)ar, (float)ai};
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < MAXE; ++q) {
        const unsigned o = threadIdx.x + q * NT;
        if (o < n) x[o] = res[q];
    }
    __syncthreads();
}

template <int CAP, bool INV>
__global__ void __launch_bounds__(NT) k_fft_any(const float2 *__restrict__ in, long long in_stride, int in_off,
                                                float2 *out, long long out_stride, int out_off, long long nrows,
                                                float scale, Plan plan) {
    constexpr int MAXE = CAP / NT;
    __shared__ float2 x[CAP];
    __shared__ float2 tw[CAP];
    const unsigned C = (unsigned)plan.C, G = (unsigned)plan.G;
    for (unsigned e = threadIdx.x; e < C; e += NT) {
        double s, c;
        sincospi(-2.0 * (double)e / (double)C, &s, &c);
        tw[e] = float2{(float)c, (float)s};
    }
    const long long ngroups = (nrows + G - 1) / G;
    for (long long grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const long long row0 = grp * G;
        for (unsigned i = threadIdx.x; i < G * C; i += NT) {
            const unsigned g = i / C, j = i - g * C;
            x[i] = row0 + g < nrows ? in[(row0 + g) * in_stride + in_off + j] : float2{0.f, 0.f};
        }
        __syncthreads();
        unsigned Lp = 1;
        for (int s = 0; s < plan.ns; ++s) {
            const unsigned p = (unsigned)plan.p[s];
            switch (p) {
            case 2: stage_small<2, MAXE, INV>(x, tw, C, G, Lp); break;
            case 3: stage_small<3, MAXE, INV>(x, tw, C, G, Lp); break;
            case 4: stage_small<4, MAXE, INV>(x, tw, C, G, Lp); break;
            case 5: stage_small<5, MAXE, INV>(x, tw, C, G, Lp); break;
            case 7: stage_small<7, MAXE, INV>(x, tw, C, G, Lp); break;
            case 8: stage_small<8, MAXE, INV>(x, tw, C, G, Lp); break;
            default: stage_any<MAXE, INV>(x, tw, C, G, Lp, p); break;
            }
            Lp *= p;
        }
        for (unsigned i = threadIdx.x; i < G * C; i += NT) {
            const unsigned g = i / C, j = i - g * C;
            if (row0 + g < nrows) {
                const float2 v = x[i];
                out[(row0 + g) * out_stride + out_off + j] = float2{v.x * scale, v.y * scale};
            }
        }
        __syncthreads();  // the next group's loads overwrite x
    }
}

// radices in stage order: 8s, then 4, 2, then the odd primes ascending
bool make_plan(int C, Plan &pl) {
    if (C < 2 || C > FFT_ANY_MAX) return false;
    pl.C = C;
    pl.G = C <= 4096 ? 4096 / C : 1;
    pl.ns = 0;
    int n = C;
    auto push = [&](int p) {
        if (pl.ns >= MAX_STAGES) return false;
        pl.p[pl.ns++] = p;
        n /= p;
        return true;
    };
    while (n % 8 == 0)
        if (!push(8)) return false;
    if (n % 4 == 0 && !push(4)) return false;
    if (n % 2 == 0 && !push(2)) return false;
    for (int p = 3; n > 1; p += 2)
        while (n % p == 0)
            if (!push(p)) return false;
    return true;
}

template <int CAP>
hipError_t launch_t(const float2 *in, long long in_stride, int in_off, float2 *out, long long out_stride,
                    int out_off, long long nrows, bool inverse, float scale, const Plan &pl, hipStream_t s) {
    const long long groups = (nrows + pl.G - 1) / pl.G;
    const unsigned grid = (unsigned)(groups < 2048 ? groups : 2048);  // persistent over the row groups
    if (inverse)
        hipLaunchKernelGGL((k_fft_any<CAP, true>), dim3(grid), dim3(NT), 0, s, in, in_stride, in_off, out,
                           out_stride, out_off, nrows, scale, pl);
    else
        hipLaunchKernelGGL((k_fft_any<CAP, false>), dim3(grid), dim3(NT), 0, s, in, in_stride, in_off, out,
                           out_stride, out_off, nrows, scale, pl);
    return hipGetLastError();
}

}  // namespace fany

bool fft_any_supported(int C) {
    fany::Plan pl;
    return fany::make_plan(C, pl);
}

hipError_t launch_fft_any(const float2 *in, long long in_stride, int in_off, float2 *out, long long out_stride,
                          int out_off, long long nrows, int C, bool inverse, float scale, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    fany::Plan pl;
    if (!fany::make_plan(C, pl)) return hipErrorInvalidValue;
    if (C <= 4096)
        return fany::launch_t<4096>(in, in_stride, in_off, out, out_stride, out_off, nrows, inverse, scale, pl, s);
    return fany::launch_t<8192>(in, in_stride, in_off, out, out_stride, out_off, nrows, inverse, scale, pl, s);
}

}  // namespace ofdm
