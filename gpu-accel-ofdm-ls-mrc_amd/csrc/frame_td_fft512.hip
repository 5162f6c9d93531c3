// frame_td_fft512.hip -- fused receivers for the FFT sizes built on one
// in-register FFT512 per wave: C = 1536 (LTE's 15 MHz size), 3072 (a wave
// pair), 6144 (a wave quad) and 512 itself.  One HBM pass over the IQ, as the
// power-of-two receivers (demodOneFrameCUDA, gpuLS.cu:575-675, without its
// cuFFT round trips), replacing the generic any-C kernel (fft_any.hip) at
// these sizes.
//
// C = 1536: one 64-lane wave transforms one antenna row held in registers,
// 24 samples per lane (lane t: x[t + 64 m'], m' < 24):
//   * radix-3 decimation in frequency in registers: for n = t + 64 m (m < 8)
//     u_j[n] = W1536^{n j} sum_i x[n + 512 i] W3^{i j},  j < 3,
//     so that X[3 k + j] = FFT512(u_j)[k];
//   * each FFT512 as 8 x 8 x 8 with two wave-local LDS transposes: pass A a
//     DFT8 over m per lane (then W512^{t s}), transpose, pass B1 a DFT8 over b
//     (t = a + 8 b; then W64^{a c}), transpose, pass B2 a DFT8 over a:
//     lane L = 8 s + c ends with X512[s + 8 c + 64 d], d < 8;
//   * packed f32 complex arithmetic (pk.hpp); the per-lane twiddles of passes
//     A and B1 are row invariants held in registers, the DIF twiddles come
//     from a W1536 table in LDS.
// Lane L therefore owns the 24 bins 3 (s + 8 c + 64 d) + j, slot i = 8 j + d.
// The channel estimate is kept in that "lane order" (k_ls_1536 writes it:
// per (frame, antenna) slot i of lane L at i * 64 + L, one coalesced 512-B
// wave load per slot); P stays bin-indexed [F][C].  A wave owns one data
// symbol at a time and walks its R rows in order (matrixMultThenSum order,
// cpuLS.hpp:187-208), the next row's 24 samples in flight during the current
// row's transform; no workgroup barrier after the table fill.
#include "common.hpp"
#include "launch.hpp"
#include "pk.hpp"

namespace ofdm {
namespace td1536 {

using pk::v2f;
constexpr int C = 1536, K = C - 1;
constexpr int PA = 72;               // transpose image: 8 rows of 64 + 8 (conflict-free reads)
constexpr int TS = 8 * PA;           // per-wave image, 4.5 KiB
constexpr int WAVES = 4;
constexpr int NT = 64 * WAVES;

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// IQ samples are streamed once: non-temporal loads keep the L2 for the
// per-frame channel estimates every data symbol of the frame re-reads.
__device__ __forceinline__ float2 ld_stream(const float2 *p) {
    return __builtin_bit_cast(float2, __builtin_nontemporal_load(reinterpret_cast<const unsigned long long *>(p)));
}

// bin of lane L's slot i (i = 8 j + d)
__device__ __forceinline__ int bin_of(int L, int i) {
    return 3 * ((L >> 3) + 8 * (L & 7) + 64 * (i & 7)) + (i >> 3);
}

// The two FFT64 passes of fft512: lane t holds v[s] = A_s[t] (8 sequences of
// 64 over the lanes) -> lane L = 8 s + c holds v[d] = FFT64(A_s)[c + 8 d].
__device__ __forceinline__ void fft64x8(v2f (&v)[8], float2 *T, int L, const v2f (&twB)[7]) {
    wsync();
#pragma unroll
    for (int s = 0; s < 8; ++s) T[s * PA + L] = pk::F(v[s]);
    wsync();
    const int s = L >> 3, a = L & 7;
#pragma unroll
    for (int b = 0; b < 8; ++b) v[b] = pk::V(T[s * PA + a + 8 * b]);
    pk::fft_reg<8>(v);  // over b -> c
#pragma unroll
    for (int c = 1; c < 8; ++c) v[c] = pk::cmul(v[c], twB[c - 1]);
    wsync();
#pragma unroll
    for (int c = 0; c < 8; ++c) T[s * PA + 9 * c + a] = pk::F(v[c]);
    wsync();
    const int c = L & 7;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = pk::V(T[s * PA + 9 * c + q]);
    pk::fft_reg<8>(v);  // over a -> d
}

// FFT512 of v (lane t: v[m] = u[t + 64 m]) -> v[d] = U[s + 8 c + 64 d], L = 8 s + c
__device__ __forceinline__ void fft512(v2f (&v)[8], float2 *T, int L, const v2f (&twA)[7], const v2f (&twB)[7]) {
    pk::fft_reg<8>(v);  // over m -> s
#pragma unroll
    for (int s = 1; s < 8; ++s) v[s] = pk::cmul(v[s], twA[s - 1]);
    fft64x8(v, T, L, twB);
}

__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_mrc_td1536(const float2 *__restrict__ iq, long long nframes, int S, int R, int prefix, const float2 *__restrict__ Hl,
             const float *__restrict__ P, float2 *__restrict__ out, int mode) {
    __shared__ float2 tab[C];             // W1536^e
    __shared__ float2 img[WAVES][TS];     // per-wave transpose images
    for (int e = threadIdx.x; e < C; e += NT) {
        double sn, cs;
        sincospi(-2.0 * (double)e / (double)C, &sn, &cs);
        tab[e] = float2{(float)cs, (float)sn};
    }
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;  // w uniform: q, f, row pointers scalar
    float2 *T = img[w];
    // row invariants: W512^{t s} = W1536^{3 t s} (t = L), W64^{a c} = W1536^{24 a c} (a = L & 7)
    v2f twA[7], twB[7];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        twA[k - 1] = pk::V(tab[(3 * L * k) % C]);
        twB[k - 1] = pk::V(tab[(24 * (L & 7) * k) % C]);
    }
    const int nsd = S - 1;
    const long long Cp = C + prefix, nq = nframes * nsd, nw = (long long)gridDim.x * WAVES;
    const float r3 = 0.86602540378443865f;  // sin(2 pi / 3)
    auto row_ptr = [&](long long q, int r) {
        const long long f = q / nsd, s = 1 + q % nsd;
        return iq + ((f * S + s) * R + r) * Cp + prefix;
    };
    float2 x[24];
    long long q = (long long)blockIdx.x * WAVES + w;
    if (q < nq) {
        const float2 *b = row_ptr(q, 0);
#pragma unroll
        for (int m = 0; m < 24; ++m) x[m] = ld_stream(b + L + 64 * m);
    }
    for (; q < nq; q += nw) {
        const long long f = q / nsd;
        // this symbol's antenna rows and the next symbol's first row: one division per symbol
        const float2 *cur = row_ptr(q, 0), *nxt = q + nw < nq ? row_ptr(q + nw, 0) : nullptr;
        v2f acc[24];
#pragma unroll
        for (int i = 0; i < 24; ++i) acc[i] = v2f{0.f, 0.f};
        for (int r = 0; r < R; ++r) {
            // radix-3 DIF in registers
            v2f u[3][8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const v2f a0 = pk::V(x[m]), a1 = pk::V(x[m + 8]), a2 = pk::V(x[m + 16]);
                const v2f sm = a1 + a2, df = a1 - a2;
                const v2f t0 = a0 - sm * (v2f){0.5f, 0.5f};
                const v2f jd = v2f{df.y * r3, -df.x * r3};  // -i sin(2 pi/3) (a1 - a2)
                const int n = L + 64 * m;
                u[0][m] = a0 + sm;
                u[1][m] = pk::cmul(t0 + jd, pk::V(tab[n]));
                u[2][m] = pk::cmul(t0 - jd, pk::V(tab[2 * n]));
            }
            // the next row (or the next symbol's first) in flight during the transforms
            {
                const float2 *b = r + 1 < R ? cur + (r + 1) * Cp : nxt;
                if (b) {
#pragma unroll
                    for (int m = 0; m < 24; ++m) x[m] = ld_stream(b + L + 64 * m);
                }
            }
            const float2 *hrow = Hl + (f * R + r) * (long long)C;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                v2f h[8];
#pragma unroll
                for (int d = 0; d < 8; ++d) h[d] = pk::V(hrow[(8 * j + d) * 64 + L]);
                fft512(u[j], T, L, twA, twB);
#pragma unroll
                for (int d = 0; d < 8; ++d) pk::mac(acc[8 * j + d], u[j][d], h[d]);
            }
        }
        float2 *o = out + q * K;
        const float *Pf = P + f * C;
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int b = bin_of(L, i);
            if (b == 0) continue;  // the DC bin carries no subcarrier
            const float2 a = pk::F(acc[i]);
            if (mode == 0) {
                const float p = Pf[b];
                o[out_pos(b - 1, K)] = float2{a.x * __builtin_amdgcn_rcpf(p), a.y * __builtin_amdgcn_rcpf(p)};
            } else {
                o[b - 1] = a;
            }
        }
    }
}

// LS from the FFT'd pilot rows (staging, bin order, frame stride R C):
// Hc = conj(Y / X) in lane order, P = sum_r |Hc|^2 (rows in order, bin layout
// with P[0] = 1 and a zero DC estimate), findHs + findDistSqrd
// (gpuLS.cu:158-209, cpuLS.hpp:211-244) as k_ls_freq.
__global__ void __launch_bounds__(256) k_ls_1536(const float2 *__restrict__ Y, int R, const float2 *__restrict__ X,
                                                 float2 *__restrict__ Hl, float *__restrict__ P) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= C) return;
    const long long f = blockIdx.y;
    const int k = b / 3, j = b - 3 * k, L = 8 * (k & 7) + ((k >> 3) & 7), i = 8 * j + (k >> 6);
    const float2 *Yf = Y + f * (long long)R * C;
    float2 *Hf = Hl + f * (long long)R * C + i * 64 + L;
    float p = 0.f;
    if (b == 0) {
        for (int r = 0; r < R; ++r) Hf[(long long)r * C] = float2{0.f, 0.f};
        p = 1.f;
    } else {
        const float2 x = X[b - 1];
        for (int r = 0; r < R; ++r) {
            const float2 h = ls_conj(Yf[(long long)r * C + b], x);
            Hf[(long long)r * C] = h;
            p = (r == 0) ? (h.x * h.x) + (h.y * h.y) : p + (h.x * h.x) + (h.y * h.y);
        }
    }
    P[f * C + b] = p;
}

}  // namespace td1536

// ---------------------------------------------------------------------------
// C = 3072 (3 x 1024: NR's 3072-point FFT) on a wave PAIR per data symbol,
// built from the same pieces: the radix-3 DIF in registers (each wave holds
// n = t + 64 (m + 8 e), m < 8, of the first 1024 and its two partners n + 1024,
// n + 2048: 24 samples per lane), then one radix-2 DIF step of the three
// FFT1024s across the pair through LDS (v0 = u[n'] + u[n' + 512] on wave 0,
// v1 = (u[n'] - u[n' + 512]) W1024^{n'} on wave 1), then three FFT512s per
// wave (td1536::fft512).  Wave e, lane 8 s + c owns bins 3 (2 k' + e) + j,
// k' = s + 8 c + 64 d, slot i = 8 j + d; the estimate in that lane order is
// [e][slot][lane] per antenna row (k_ls_3072).  Two LDS barriers per row (the
// exchange written / read); the exchange image of a wave doubles as its
// transpose image once both have read it.
namespace td3072 {

using pk::v2f;
constexpr int C = 3072, K = C - 1;
constexpr int XS = 24 * 64;  // exchange image per wave (float2): [j][m][t]
constexpr int NT = 128;      // one pair per workgroup
static_assert(td1536::TS <= XS, "transpose image fits in the exchange image");

__device__ __forceinline__ void pair_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int bin_of(int e, int L, int i) {
    return 3 * (2 * ((L >> 3) + 8 * (L & 7) + 64 * (i & 7)) + e) + (i >> 3);
}

__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_mrc_td3072(const float2 *__restrict__ iq, long long nframes, int S, int R, int prefix, const float2 *__restrict__ Hl,
             const float *__restrict__ P, float2 *__restrict__ out, int mode) {
    __shared__ float2 tab[2048];   // W3072^e, e < 2048 (DIF twiddles n j, n < 1024, j <= 2)
    __shared__ float2 xch[2][XS];  // per-wave exchange / transpose image
    for (int e = threadIdx.x; e < 2048; e += NT) {
        double sn, cs;
        sincospi(-2.0 * (double)e / (double)C, &sn, &cs);
        tab[e] = float2{(float)cs, (float)sn};
    }
    const int e = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;
    v2f twA[7], twB[7];  // W512^{t s}, W64^{a c}: the FFT512 row invariants
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        double sn, cs;
        sincospi(-2.0 * (double)((L * k) % 512) / 512.0, &sn, &cs);
        twA[k - 1] = v2f{(float)cs, (float)sn};
        sincospi(-2.0 * (double)(((L & 7) * k) % 64) / 64.0, &sn, &cs);
        twB[k - 1] = v2f{(float)cs, (float)sn};
    }
    __syncthreads();
    float2 *own = xch[e], *oth = xch[e ^ 1];
    const int nsd = S - 1;
    const long long Cp = C + prefix, nq = nframes * nsd, np = gridDim.x;
    const float r3 = 0.86602540378443865f;
    auto row_ptr = [&](long long q, int r) {
        const long long f = q / nsd, s = 1 + q % nsd;
        return iq + ((f * S + s) * R + r) * Cp + prefix;
    };
    // lane L of wave e loads x[L + 64 (m + 8 e + 16 i)], m < 8, i < 3, into x[8 i + m]
    auto load = [&](float2 (&x)[24], const float2 *b) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int m = 0; m < 8; ++m) x[8 * i + m] = td1536::ld_stream(b + L + 64 * (m + 8 * e + 16 * i));
    };
    float2 x[24];
    long long q = blockIdx.x;
    if (q < nq) load(x, row_ptr(q, 0));
    for (; q < nq; q += np) {
        const long long f = q / nsd;
        const float2 *cur = row_ptr(q, 0), *nxt = q + np < nq ? row_ptr(q + np, 0) : nullptr;
        v2f acc[24];
#pragma unroll
        for (int i = 0; i < 24; ++i) acc[i] = v2f{0.f, 0.f};
        for (int r = 0; r < R; ++r) {
            v2f u[3][8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const v2f a0 = pk::V(x[m]), a1 = pk::V(x[m + 8]), a2 = pk::V(x[m + 16]);
                const v2f sm = a1 + a2, df = a1 - a2;
                const v2f t0 = a0 - sm * (v2f){0.5f, 0.5f};
                const v2f jd = v2f{df.y * r3, -df.x * r3};
                const int n = L + 64 * (m + 8 * e);
                u[0][m] = a0 + sm;
                u[1][m] = pk::cmul(t0 + jd, pk::V(tab[n]));
                u[2][m] = pk::cmul(t0 - jd, pk::V(tab[2 * n]));
            }
            {
                const float2 *b = r + 1 < R ? cur + (r + 1) * Cp : nxt;
                if (b) load(x, b);
            }
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int m = 0; m < 8; ++m) own[(8 * j + m) * 64 + L] = pk::F(u[j][m]);
            pair_barrier();
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const v2f p = pk::V(oth[(8 * j + m) * 64 + L]);
                    // wave 0: u[n'] + u[n' + 512]; wave 1: (u[n'] - u[n' + 512]) W1024^{n'}, n' = L + 64 m
                    u[j][m] = e == 0 ? u[j][m] + p : pk::cmul(p - u[j][m], pk::V(tab[3 * (L + 64 * m)]));
                }
            pair_barrier();  // both exchange images read: each becomes its wave's transpose image
            const float2 *hrow = Hl + (f * R + r) * (long long)C + e * 1536;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                v2f h[8];
#pragma unroll
                for (int d = 0; d < 8; ++d) h[d] = pk::V(hrow[(8 * j + d) * 64 + L]);
                td1536::fft512(u[j], own, L, twA, twB);
#pragma unroll
                for (int d = 0; d < 8; ++d) pk::mac(acc[8 * j + d], u[j][d], h[d]);
            }
        }
        float2 *o = out + q * K;
        const float *Pf = P + f * C;
        // the lane recomputed here: output offsets hoisted out of the symbol
        // loop were spilled and reloaded behind a vmcnt(0) that drained the
        // next symbol's row load
        const int Le = lane_here();
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int b = bin_of(e, Le, i);
            if (b == 0) continue;
            const float2 a = pk::F(acc[i]);
            if (mode == 0) {
                const float p = Pf[b];
                o[out_pos(b - 1, K)] = float2{a.x * __builtin_amdgcn_rcpf(p), a.y * __builtin_amdgcn_rcpf(p)};
            } else {
                o[b - 1] = a;
            }
        }
    }
}

// LS into the lane order of k_mrc_td3072 ([e][slot][lane] per antenna row)
__global__ void __launch_bounds__(256) k_ls_3072(const float2 *__restrict__ Y, int R, const float2 *__restrict__ X,
                                                 float2 *__restrict__ Hl, float *__restrict__ P) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= C) return;
    const long long f = blockIdx.y;
    const int k = b / 3, j = b - 3 * k, kk = k >> 1, e = k & 1;
    const int L = 8 * (kk & 7) + ((kk >> 3) & 7), i = 8 * j + (kk >> 6);
    const float2 *Yf = Y + f * (long long)R * C;
    float2 *Hf = Hl + f * (long long)R * C + e * 1536 + i * 64 + L;
    float p = 0.f;
    if (b == 0) {
        for (int r = 0; r < R; ++r) Hf[(long long)r * C] = float2{0.f, 0.f};
        p = 1.f;
    } else {
        const float2 x = X[b - 1];
        for (int r = 0; r < R; ++r) {
            const float2 h = ls_conj(Yf[(long long)r * C + b], x);
            Hf[(long long)r * C] = h;
            p = (r == 0) ? (h.x * h.x) + (h.y * h.y) : p + (h.x * h.x) + (h.y * h.y);
        }
    }
    P[f * C + b] = p;
}

}  // namespace td3072

// ---------------------------------------------------------------------------
// C = 6144 (3 x 2048) on a wave QUAD per data symbol: the radix-3 DIF in
// registers (wave e holds n = t + 64 (m + 8 e) < 2048 and its partners
// n + 2048, n + 4096), one radix-4 DIF step of the three FFT2048s across the
// quad through LDS (wave e forms branch e: v_e[n'] = W2048^{n' e}
// sum_h u[n' + 512 h] W4^{h e}, n' = t + 64 m), then three FFT512s per wave.
// Wave e, lane 8 s + c owns bins 3 (4 k' + e) + j, k' = s + 8 c + 64 d; the
// estimate is [e][slot][lane] per row (k_ls_6144).
namespace td6144 {

using pk::v2f;
constexpr int C = 6144, K = C - 1;
constexpr int XS = 24 * 64;
constexpr int NT = 256;  // one quad per workgroup

__device__ __forceinline__ int bin_of(int e, int L, int i) {
    return 3 * (4 * ((L >> 3) + 8 * (L & 7) + 64 * (i & 7)) + e) + (i >> 3);
}

__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_mrc_td6144(const float2 *__restrict__ iq, long long nframes, int S, int R, int prefix, const float2 *__restrict__ Hl,
             const float *__restrict__ P, float2 *__restrict__ out, int mode) {
    __shared__ float2 tab[4096];   // W6144^e, e < 4096 (e >= 4096: -W6144^{e - 3072}); every twiddle one table entry
    __shared__ float2 xch[4][XS];  // per-wave exchange / transpose image
    static_assert((4096 + 4 * XS) * sizeof(float2) <= 80 * 1024, "two workgroups per CU (160 KiB of LDS)");
    for (int e = threadIdx.x; e < 4096; e += NT) {
        double sn, cs;
        sincospi(-2.0 * (double)e / (double)C, &sn, &cs);
        tab[e] = float2{(float)cs, (float)sn};
    }
    const int e = threadIdx.x >> 6, L = threadIdx.x & 63;
    v2f twA[7], twB[7];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        double sn, cs;
        sincospi(-2.0 * (double)((L * k) % 512) / 512.0, &sn, &cs);
        twA[k - 1] = v2f{(float)cs, (float)sn};
        sincospi(-2.0 * (double)(((L & 7) * k) % 64) / 64.0, &sn, &cs);
        twB[k - 1] = v2f{(float)cs, (float)sn};
    }
    __syncthreads();
    float2 *own = xch[e];
    const int nsd = S - 1;
    const long long Cp = C + prefix, nq = nframes * nsd, np = gridDim.x;
    const float r3 = 0.86602540378443865f;
    auto row_ptr = [&](long long q, int r) {
        const long long f = q / nsd, s = 1 + q % nsd;
        return iq + ((f * S + s) * R + r) * Cp + prefix;
    };
    auto load = [&](float2 (&x)[24], const float2 *b) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int m = 0; m < 8; ++m) x[8 * i + m] = td1536::ld_stream(b + L + 64 * (m + 8 * e + 32 * i));
    };
    float2 x[24];
    long long q = blockIdx.x;
    if (q < nq) load(x, row_ptr(q, 0));
    for (; q < nq; q += np) {
        const long long f = q / nsd;
        v2f acc[24];
#pragma unroll
        for (int i = 0; i < 24; ++i) acc[i] = v2f{0.f, 0.f};
        for (int r = 0; r < R; ++r) {
            v2f u[3][8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const v2f a0 = pk::V(x[m]), a1 = pk::V(x[m + 8]), a2 = pk::V(x[m + 16]);
                const v2f sm = a1 + a2, df = a1 - a2;
                const v2f t0 = a0 - sm * (v2f){0.5f, 0.5f};
                const v2f jd = v2f{df.y * r3, -df.x * r3};
                const int n = L + 64 * (m + 8 * e);
                u[0][m] = a0 + sm;
                u[1][m] = pk::cmul(t0 + jd, pk::V(tab[n]));
                u[2][m] = pk::cmul(t0 - jd, pk::V(tab[2 * n]));  // 2 n < 4096
            }
            {
                const long long qn = r + 1 < R ? q : q + np;
                if (qn < nq) load(x, row_ptr(qn, r + 1 < R ? r + 1 : 0));
            }
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int m = 0; m < 8; ++m) own[(8 * j + m) * 64 + L] = pk::F(u[j][m]);
            td3072::pair_barrier();
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                // W2048^{n' e} = W6144^{3 n' e}, n' = L + 64 m (3 n' e < 4608; W6144^{x + 3072} = -W6144^x)
                const int x3 = 3 * (L + 64 * m) * e;
                const v2f we = x3 < 4096 ? pk::V(tab[x3]) : -pk::V(tab[x3 - 3072]);
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const v2f h0 = pk::V(xch[0][(8 * j + m) * 64 + L]), h1 = pk::V(xch[1][(8 * j + m) * 64 + L]);
                    const v2f h2 = pk::V(xch[2][(8 * j + m) * 64 + L]), h3 = pk::V(xch[3][(8 * j + m) * 64 + L]);
                    // sum_h u[n' + 512 h] W4^{h e}, W4 = -i
                    const v2f s02 = h0 + h2, d02 = h0 - h2, s13 = h1 + h3, d13 = h1 - h3;
                    const v2f md13 = v2f{d13.y, -d13.x};  // -i (h1 - h3)
                    v2f v = e == 0 ? s02 + s13 : e == 1 ? d02 + md13 : e == 2 ? s02 - s13 : d02 - md13;
                    u[j][m] = e == 0 ? v : pk::cmul(v, we);
                }
            }
            td3072::pair_barrier();
            const float2 *hrow = Hl + (f * R + r) * (long long)C + e * 1536;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                v2f h[8];
#pragma unroll
                for (int d = 0; d < 8; ++d) h[d] = pk::V(hrow[(8 * j + d) * 64 + L]);
                td1536::fft512(u[j], own, L, twA, twB);
#pragma unroll
                for (int d = 0; d < 8; ++d) pk::mac(acc[8 * j + d], u[j][d], h[d]);
            }
        }
        float2 *o = out + q * K;
        const float *Pf = P + f * C;
        // the lane recomputed here: output offsets hoisted out of the symbol
        // loop were spilled and reloaded behind a vmcnt(0) that drained the
        // next symbol's row load
        const int Le = lane_here();
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int b = bin_of(e, Le, i);
            if (b == 0) continue;
            const float2 a = pk::F(acc[i]);
            if (mode == 0) {
                const float p = Pf[b];
                o[out_pos(b - 1, K)] = float2{a.x * __builtin_amdgcn_rcpf(p), a.y * __builtin_amdgcn_rcpf(p)};
            } else {
                o[b - 1] = a;
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_ls_6144(const float2 *__restrict__ Y, int R, const float2 *__restrict__ X,
                                                 float2 *__restrict__ Hl, float *__restrict__ P) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= C) return;
    const long long f = blockIdx.y;
    const int k = b / 3, j = b - 3 * k, kk = k >> 2, e = k & 3;  // b = 3 (4 k' + e) + j
    const int L = 8 * (kk & 7) + ((kk >> 3) & 7), i = 8 * j + (kk >> 6);
    const float2 *Yf = Y + f * (long long)R * C;
    float2 *Hf = Hl + f * (long long)R * C + e * 1536 + i * 64 + L;
    float p = 0.f;
    if (b == 0) {
        for (int r = 0; r < R; ++r) Hf[(long long)r * C] = float2{0.f, 0.f};
        p = 1.f;
    } else {
        const float2 x = X[b - 1];
        for (int r = 0; r < R; ++r) {
            const float2 h = ls_conj(Yf[(long long)r * C + b], x);
            Hf[(long long)r * C] = h;
            p = (r == 0) ? (h.x * h.x) + (h.y * h.y) : p + (h.x * h.x) + (h.y * h.y);
        }
    }
    P[f * C + b] = p;
}

}  // namespace td6144

// ---------------------------------------------------------------------------
// C = 512, 256, 128 (LTE's 5, 3 and 1.4 MHz sizes; 512 is also the FFT of the
// receivers above): one wave per data symbol, NR = 512 / C antenna rows per
// pass, P = C / 64 samples of each per lane (lane t: v[rho P + m] =
// x_{r0 + rho}[t + 64 m], m < P).  Pass A is a DFT_P per row with W_C^{t s'};
// the NR P = 8 sequences then go through fft512's two FFT64 passes unchanged,
// so lane L = 8 (rho P + s') + c ends with bins s' + P c + 8 P d (slot d) of
// row r0 + rho.  Each lane accumulates its rows rho, rho + NR, ...; the NR
// partial sums meet once per symbol (lane xor 8 P, 16 P).  Estimate per row:
// [slot d][lane mod 8 P] (k_ls_small).  Rows past R enter as zeros.
namespace tdsmall {

using pk::v2f;
constexpr int WAVES = 4, NT = 64 * WAVES;

template <int NR>
__device__ __forceinline__ void mrc_small(const float2 *__restrict__ iq, long long nframes, int S, int R, int prefix,
                                          const float2 *__restrict__ Hl, const float *__restrict__ P,
                                          float2 *__restrict__ out, int mode) {
    constexpr int NP = 8 / NR, C = 64 * NP, K = C - 1, LW = 8 * NP;
    __shared__ float2 img[WAVES][td1536::TS];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63, rho = L / LW, lw = L % LW;
    float2 *T = img[w];
    v2f twA[NP > 1 ? NP - 1 : 1], twB[7];
#pragma unroll
    for (int k = 1; k < NP; ++k) {
        double sn, cs;
        sincospi(-2.0 * (double)((L * k) % C) / (double)C, &sn, &cs);
        twA[k - 1] = v2f{(float)cs, (float)sn};
    }
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        double sn, cs;
        sincospi(-2.0 * (double)(((L & 7) * k) % 64) / 64.0, &sn, &cs);
        twB[k - 1] = v2f{(float)cs, (float)sn};
    }
    const int nsd = S - 1;
    const long long Cp = C + prefix, nq = nframes * nsd, nw = (long long)gridDim.x * WAVES;
    float2 x[8];
    auto row_ptr = [&](long long qq) {  // antenna row 0 of data symbol qq
        const long long f = qq / nsd, s = 1 + qq % nsd;
        return iq + (f * S + s) * R * Cp + prefix;
    };
    auto load = [&](const float2 *b, int r0) {  // rows r0 .. r0 + NR - 1 from row r0 at b (wave-uniform)
#pragma unroll
        for (int g = 0; g < NR; ++g)
#pragma unroll
            for (int m = 0; m < NP; ++m) x[g * NP + m] = r0 + g < R ? td1536::ld_stream(b + g * Cp + L + 64 * m) : float2{0.f, 0.f};
    };
    long long q = (long long)blockIdx.x * WAVES + w;
    if (q < nq) load(row_ptr(q), 0);
    for (; q < nq; q += nw) {
        const long long f = q / nsd;
        const float2 *cur = row_ptr(q), *nxt = q + nw < nq ? row_ptr(q + nw) : nullptr;
        v2f acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = v2f{0.f, 0.f};
        for (int r0 = 0; r0 < R; r0 += NR) {
            v2f u[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) u[m] = pk::V(x[m]);
            {
                const float2 *b = r0 + NR < R ? cur + (r0 + NR) * Cp : nxt;
                if (b) load(b, r0 + NR < R ? r0 + NR : 0);
            }
            // this lane's row; a row past R has zero samples, its (clamped) estimate multiplies zeros
            const int r = r0 + rho < R ? r0 + rho : R - 1;
            const float2 *hrow = Hl + (f * R + r) * (long long)C + lw;
            v2f h[8];
#pragma unroll
            for (int d = 0; d < 8; ++d) h[d] = pk::V(hrow[d * LW]);
#pragma unroll
            for (int g = 0; g < NR; ++g) {  // pass A: DFT_P per row, then W_C^{t s'}
                v2f a[NP];
#pragma unroll
                for (int m = 0; m < NP; ++m) a[m] = u[g * NP + m];
                pk::fft_reg<NP>(a);
#pragma unroll
                for (int k = 1; k < NP; ++k) a[k] = pk::cmul(a[k], twA[k - 1]);
#pragma unroll
                for (int m = 0; m < NP; ++m) u[g * NP + m] = a[m];
            }
            td1536::fft64x8(u, T, L, twB);
#pragma unroll
            for (int d = 0; d < 8; ++d) pk::mac(acc[d], u[d], h[d]);
        }
#pragma unroll
        for (int o = LW; o < 64; o <<= 1)
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                const float2 a = pk::F(acc[d]);
                acc[d] += v2f{__shfl_xor(a.x, o), __shfl_xor(a.y, o)};
            }
        if (rho != 0) continue;
        float2 *o = out + q * K;
        const float *Pf = P + f * C;
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const int b = (lw >> 3) + NP * (lw & 7) + LW * d;
            if (b == 0) continue;  // the DC bin carries no subcarrier
            const float2 a = pk::F(acc[d]);
            if (mode == 0) {
                const float p = Pf[b];
                o[out_pos(b - 1, K)] = float2{a.x * __builtin_amdgcn_rcpf(p), a.y * __builtin_amdgcn_rcpf(p)};
            } else {
                o[b - 1] = a;
            }
        }
    }
}

// LS from the FFT'd pilot rows into the lane order above (as k_ls_1536).
template <int NR>
__device__ __forceinline__ void ls_small(const float2 *__restrict__ Y, int R, const float2 *__restrict__ X,
                                         float2 *__restrict__ Hl, float *__restrict__ P) {
    constexpr int NP = 8 / NR, C = 64 * NP, LW = 8 * NP;
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= C) return;
    const long long f = blockIdx.y;
    const int pos = (b / LW) * LW + 8 * (b % NP) + ((b / NP) & 7);
    const float2 *Yf = Y + f * (long long)R * C;
    float2 *Hf = Hl + f * (long long)R * C + pos;
    float p = 0.f;
    if (b == 0) {
        for (int r = 0; r < R; ++r) Hf[(long long)r * C] = float2{0.f, 0.f};
        p = 1.f;
    } else {
        const float2 x = X[b - 1];
        for (int r = 0; r < R; ++r) {
            const float2 h = ls_conj(Yf[(long long)r * C + b], x);
            Hf[(long long)r * C] = h;
            p = (r == 0) ? (h.x * h.x) + (h.y * h.y) : p + (h.x * h.x) + (h.y * h.y);
        }
    }
    P[f * C + b] = p;
}

#define OFDM_TD_SMALL(CC, NR)                                                                                          \
    __global__ void __launch_bounds__(NT) k_mrc_td##CC(const float2 *__restrict__ iq, long long nframes, int S, int R, \
                                                       int prefix, const float2 *__restrict__ Hl,                      \
                                                       const float *__restrict__ P, float2 *__restrict__ out,          \
                                                       int mode) {                                                     \
        mrc_small<NR>(iq, nframes, S, R, prefix, Hl, P, out, mode);                                                    \
    }                                                                                                                  \
    __global__ void __launch_bounds__(256) k_ls_##CC(const float2 *__restrict__ Y, int R,                              \
                                                     const float2 *__restrict__ X, float2 *__restrict__ Hl,            \
                                                     float *__restrict__ P) {                                          \
        ls_small<NR>(Y, R, X, Hl, P);                                                                                  \
    }
OFDM_TD_SMALL(512, 1)
OFDM_TD_SMALL(256, 2)
OFDM_TD_SMALL(128, 4)
#undef OFDM_TD_SMALL

}  // namespace tdsmall

namespace {

int cu_count() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return cus;
}

// One workgroup column per 256 bins, one grid row per frame (65535 at a time).
template <int CC, typename Kern>
hipError_t launch_ls_lane(Kern kern, const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                          hipStream_t s) {
    if (nframes <= 0) return hipSuccess;
    for (long long f0 = 0; f0 < nframes; f0 += 65535) {
        const long long n = nframes - f0 < 65535 ? nframes - f0 : 65535;
        hipLaunchKernelGGL(kern, dim3((CC + 255) / 256, (unsigned)n), dim3(256), 0, s, Y + f0 * (long long)R * CC, R,
                           X, Hl + f0 * (long long)R * CC, P + f0 * CC);
    }
    return hipGetLastError();
}

// Persistent grid: min(workgroups needed, per_cu x CUs); each workgroup owns
// `per_wg` data symbols at a time.
template <typename Kern>
hipError_t launch_mrc_lane(Kern kern, int nt, int per_cu, int per_wg, const float2 *iq, long long nframes, int S,
                           int R, int prefix, const float2 *Hl, const float *P, float2 *out, int mode, hipStream_t s) {
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    // the resident count from the occupancy query (LDS, registers), capped by
    // the hint: a kernel that outgrows its LDS budget shrinks the grid
    // instead of queueing workgroups behind a persistent one
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(kern), nt, 0) ==
            hipSuccess &&
        occ > 0 && occ < per_cu)
        per_cu = occ;
    const long long res = (long long)per_cu * cu_count(), need = (nq + per_wg - 1) / per_wg;
    hipLaunchKernelGGL(kern, dim3((unsigned)(need < res ? need : res)), dim3(nt), 0, s, iq, nframes, S, R, prefix, Hl,
                       P, out, mode);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_ls_small(int C, const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                           hipStream_t s) {
    return C == 512   ? launch_ls_lane<512>(tdsmall::k_ls_512, Y, nframes, R, X, Hl, P, s)
           : C == 256 ? launch_ls_lane<256>(tdsmall::k_ls_256, Y, nframes, R, X, Hl, P, s)
           : C == 128 ? launch_ls_lane<128>(tdsmall::k_ls_128, Y, nframes, R, X, Hl, P, s)
                      : hipErrorInvalidValue;
}

hipError_t launch_ls_1536(const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                          hipStream_t s) {
    return launch_ls_lane<td1536::C>(td1536::k_ls_1536, Y, nframes, R, X, Hl, P, s);
}

hipError_t launch_ls_3072(const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                          hipStream_t s) {
    return launch_ls_lane<td3072::C>(td3072::k_ls_3072, Y, nframes, R, X, Hl, P, s);
}

hipError_t launch_ls_6144(const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                          hipStream_t s) {
    return launch_ls_lane<td6144::C>(td6144::k_ls_6144, Y, nframes, R, X, Hl, P, s);
}

// 512 / 256 / 128: 4 one-wave symbols per workgroup, 4 workgroups per CU.
hipError_t launch_mrc_small(int C, const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                            const float *P, float2 *out, int mode, hipStream_t s) {
    using namespace tdsmall;
    auto kern = C == 512 ? k_mrc_td512 : C == 256 ? k_mrc_td256 : C == 128 ? k_mrc_td128 : nullptr;
    if (!kern) return hipErrorInvalidValue;
    return launch_mrc_lane(kern, NT, 4, WAVES, iq, nframes, S, R, prefix, Hl, P, out, mode, s);
}

// 1536: 4 one-wave symbols per workgroup, 2 workgroups per CU (2 waves / SIMD).
hipError_t launch_mrc_td1536(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                             const float *P, float2 *out, int mode, hipStream_t s) {
    return launch_mrc_lane(td1536::k_mrc_td1536, td1536::NT, 2, td1536::WAVES, iq, nframes, S, R, prefix, Hl, P, out,
                           mode, s);
}

// 3072: one wave pair (40 KiB of LDS) per workgroup, 4 per CU.
hipError_t launch_mrc_td3072(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                             const float *P, float2 *out, int mode, hipStream_t s) {
    return launch_mrc_lane(td3072::k_mrc_td3072, td3072::NT, 4, 1, iq, nframes, S, R, prefix, Hl, P, out, mode, s);
}

// 6144: one wave quad (80 KiB of static LDS: the 32 KiB twiddle table and
// four 12 KiB exchange images) per workgroup, 2 per CU (static_assert in
// k_mrc_td6144; the occupancy query in launch_mrc_lane has the last word).
hipError_t launch_mrc_td6144(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                             const float *P, float2 *out, int mode, hipStream_t s) {
    return launch_mrc_lane(td6144::k_mrc_td6144, td6144::NT, 2, 1, iq, nframes, S, R, prefix, Hl, P, out, mode, s);
}

}  // namespace ofdm
