// common.hpp -- device-side helpers shared by the LS/MRC kernels (gfx950).
//
// Complex values are float2 {re, im}: byte-identical to the reference's
// complexF (ShMemSymBuff.hpp:86-89) and to ofdm_cf32 in include/ofdm_lsmrc.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "twiddles.inc"  // generated: OFDM_TW_N, OFDM_TW_TABLE

namespace ofdm {

// W_4096^k = exp(-2*pi*i*k/4096), k < 4096.  Runtime-indexed copy (global
// memory, read through L1/L2) ...
__constant__ __attribute__((aligned(16))) float g_twf[2 * OFDM_TW_N] = {OFDM_TW_TABLE};
#define g_tw (reinterpret_cast<const float2 *>(g_twf))
// ... and a compile-time copy so constant-index uses fold to immediates.
struct TwTable { float v[2 * OFDM_TW_N]; };
constexpr TwTable kTw = {{OFDM_TW_TABLE}};

// W_N^k for compile-time N | 4096 and compile-time k (forward sign).
template <int N, int K>
__device__ __forceinline__ constexpr float2 tw_const() {
    static_assert(OFDM_TW_N % N == 0, "N must divide 4096");
    constexpr int idx = ((K % N + N) % N) * (OFDM_TW_N / N);
    return float2{kTw.v[2 * idx], kTw.v[2 * idx + 1]};
}

// The lane index recomputed where it is used (volatile: never merged with
// threadIdx.x nor hoisted), so that the lane and its derived values need not
// stay live (spilled to scratch) across a loop that does not use them.
__device__ __forceinline__ int lane_here() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ float2 cconj(float2 a) { return {a.x, -a.y}; }
// multiply by -i (forward) / +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 cmul_mi(float2 a) {
    return INV ? float2{-a.y, a.x} : float2{a.y, -a.x};
}
template <bool INV>
__device__ __forceinline__ float2 tw_apply(float2 a, float2 w) {
    return cmul(a, INV ? cconj(w) : w);
}

// --------------------------------------------------------------------------
// In-register radix-2 FFT of N points held by one lane (natural order in and
// out).  All indices and twiddles are compile-time; trivial twiddles (1, -i)
// are applied without multiplies.
// --------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ constexpr int bitrev(int i) {
    int r = 0;
    for (int b = 1, rb = N >> 1; b < N; b <<= 1, rb >>= 1)
        if (i & b) r |= rb;
    return r;
}

template <int N, bool INV>
__device__ __forceinline__ void fft_reg(float2 (&a)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int j = bitrev<N>(i);
        if (i < j) { float2 t = a[i]; a[i] = a[j]; a[j] = t; }
    }
#pragma unroll
    for (int len = 2; len <= N; len <<= 1) {
        const int half = len >> 1;
#pragma unroll
        for (int i = 0; i < N; i += len) {
#pragma unroll
            for (int k = 0; k < half; ++k) {
                float2 u = a[i + k], v = a[i + k + half];
                if (k == 0) {
                } else if (4 * k == len) {
                    v = cmul_mi<INV>(v);
                } else {
                    const int idx = k * (OFDM_TW_N / len);
                    float2 w{kTw.v[2 * idx], kTw.v[2 * idx + 1]};
                    v = tw_apply<INV>(v, w);
                }
                a[i + k] = cadd(u, v);
                a[i + k + half] = csub(u, v);
            }
        }
    }
}

// --------------------------------------------------------------------------
// Block-cooperative Stockham autosort FFT in LDS (radix-4 stages, one final
// radix-2 stage when log2(C) is odd).  Input in `a`, scratch `b`; returns the
// buffer holding the natural-order result.  Caller synchronises before.
// --------------------------------------------------------------------------
template <int LOG2C, bool INV>
__device__ float2 *stockham_lds(float2 *a, float2 *b) {
    constexpr int C = 1 << LOG2C;
    constexpr int TWS = OFDM_TW_N / C;
    int Ns = 1;
#pragma unroll 1
    for (; Ns * 4 <= C; Ns *= 4) {
        for (int j = threadIdx.x; j < C / 4; j += blockDim.x) {
            const int k = j & (Ns - 1);
            float2 v0 = a[j], v1 = a[j + C / 4], v2 = a[j + C / 2], v3 = a[j + 3 * C / 4];
            const int t = k * (C / (4 * Ns));
            if (t) {
                v1 = tw_apply<INV>(v1, g_tw[t * TWS]);
                v2 = tw_apply<INV>(v2, g_tw[2 * t * TWS]);
                v3 = tw_apply<INV>(v3, g_tw[3 * t * TWS]);
            }
            const float2 s02 = cadd(v0, v2), d02 = csub(v0, v2);
            const float2 s13 = cadd(v1, v3), d13 = cmul_mi<INV>(csub(v1, v3));
            const int d = (j - k) * 4 + k;
            b[d] = cadd(s02, s13);
            b[d + Ns] = cadd(d02, d13);
            b[d + 2 * Ns] = csub(s02, s13);
            b[d + 3 * Ns] = csub(d02, d13);
        }
        __syncthreads();
        float2 *t = a; a = b; b = t;
    }
    if (Ns < C) {  // final radix-2 stage, Ns == C/2
        for (int j = threadIdx.x; j < C / 2; j += blockDim.x) {
            const int k = j & (Ns - 1);
            float2 v0 = a[j], v1 = a[j + C / 2];
            const int t = k * (C / (2 * Ns));
            if (t) v1 = tw_apply<INV>(v1, g_tw[t * TWS]);
            const int d = (j - k) * 2 + k;
            b[d] = cadd(v0, v1);
            b[d + Ns] = csub(v0, v1);
        }
        __syncthreads();
        float2 *t = a; a = b; b = t;
    }
    return a;
}

// --------------------------------------------------------------------------
// Receiver index maps (K = C - 1 used subcarriers).
// Bin b = j + 1 of the FFT carries subcarrier j (DC dropped, cpuLS.hpp:290-292).
// Output position of subcarrier j after shiftOneRow (cpuLS.hpp:135-149), odd
// K (every even C, so every fused receiver and the paired-bin kernels):
//   out[k] = Z[k + (K-1)/2]        for k <  (K+1)/2
//   out[k] = Z[k - (K+1)/2]        for k >= (K+1)/2
// --------------------------------------------------------------------------
__device__ __forceinline__ int out_pos(int j, int K) {
    const int h = (K - 1) / 2;
    return j >= h ? j - h : j + (K + 1) / 2;
}
// Any K: shiftOneRow's three memmoves literally, h = (K-1)/2, n2 = (K+1)/2:
//   out[k] = Z[k + h] (k < n2),  Z[k - n2] (n2 <= k < n2 + h),  Z[k] (k >= n2 + h)
// -- for even K (odd C) the CPU reference leaves the last element in place
// (its GPU kernel, gpuLS.cu:109-125, would duplicate Z[h] there instead; the
// CPU function is the one the oracle pins).  Equal to out_pos for odd K.
__device__ __forceinline__ int out_pos_any(int j, int K) {
    const int h = (K - 1) / 2, n2 = (K + 1) / 2;
    return j < h ? j + n2 : (j < h + n2 ? j - h : j);
}
// the subcarrier that out_pos_any puts at output position k
__device__ __forceinline__ int out_src(int k, int K) {
    const int h = (K - 1) / 2, n2 = (K + 1) / 2;
    return k < n2 ? k + h : (k < n2 + h ? k - n2 : k);
}

// LS for one subcarrier: conj(y / x) with divideOneRow's naive formula
// (cpuLS.hpp:240-241) followed by the conjugate (303-307).
// The two divisions by |x|^2 as one reciprocal (v_rcp_f32, 1 ulp) and two
// products: within 2 ulp of the reference's quotients, ~18 fewer
// instructions per bin in the estimators' rows (the first round of the
// one-launch demod waits for them).
__device__ __forceinline__ float2 ls_conj(float2 y, float2 x) {
    const float den = x.x * x.x + x.y * x.y;
    const float rd = __builtin_amdgcn_rcpf(den);
    const float re = (y.x * x.x + y.y * x.y) * rd;
    const float im = (y.y * x.x - y.x * x.y) * rd;
    return {re, -1.0f * im};
}

// Deterministic counter-based RNG for synthetic frames.
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t hash4(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
    return splitmix64(splitmix64(splitmix64(seed ^ a) ^ b) ^ c);
}
__device__ __forceinline__ float u01(uint32_t x) {  // (0, 1]
    return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float2 gauss2(uint64_t h) {  // two N(0,1)
    const float u1 = u01((uint32_t)h), u2 = u01((uint32_t)(h >> 32));
    const float rad = sqrtf(-2.0f * logf(u1));
    float s, c;
    sincosf(6.283185307179586f * u2, &s, &c);
    return {rad * c, rad * s};
}

}  // namespace ofdm
