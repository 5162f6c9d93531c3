// pn_sync.hip -- PN-sequence frame synchronisation on the GPU (SURVEY.md 8(f)
// rank 3): the sliding correlator of rx_and_corr.cpp:332-360 and the frame
// extraction of rx_and_corr.cpp:370-392 + copy_to_shared_mem (64-87), so a
// received buffer can go correlate -> extract -> ofdm_frame_demod without
// leaving HBM.
//
// The correlator's output is an INDEX (the first channel/lag whose
// normalised correlation reaches the threshold), so it must agree with the
// reference bit for bit, including at lags whose value sits right at the
// threshold.  Every lag is therefore evaluated in the reference's own
// arithmetic: std::complex<float> products (ac - bd, ad + bc) summed in f32
// in sequential j order with no FMA contraction, |.| as glibc's hypotf
// (sqrt of the sum of squares in double, rounded to float), divided by
// (float)L.  That rules out FFT / MFMA formulations (different summation
// order); the kernel is a VALU-bound direct correlation:
//   * a 256-thread workgroup owns 1024 consecutive lags of one channel; each
//     wave 256 of them, four per lane at stride 64 (lane-contiguous LDS
//     reads, no bank conflicts, and every read of a 4-tap step is a constant
//     offset from one address);
//   * the samples x[i0 + j0 .. i0 + j0 + 1024 + JC) are staged in LDS per
//     chunk of JC = 1024 PN taps, with the chunk's taps (broadcast reads);
//   * early exit as in the reference's `break`: workgroups are dispatched in
//     channel-major lag order and a hit publishes its (channel, lag) key with
//     atomicMin; a workgroup whose first key is not below the best key found
//     so far stops at the next chunk boundary (the key order IS the
//     reference's search order, so the minimum is the reference's hit).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "launch.hpp"

namespace ofdm {
namespace pn {

constexpr int NT = 256;          // threads per workgroup
constexpr int LPT = 4;           // lags per thread
constexpr int TILE = NT * LPT;   // lags per workgroup
constexpr int JC = 1024;         // PN taps per LDS chunk

#pragma clang fp contract(off)

typedef float v2f __attribute__((ext_vector_type(2)));

// acc += p * v in the reference's exact operations, packed: each VOP3P
// instruction does the same IEEE f32 operation on both halves, op_sel /
// op_sel_hi pick the halves and neg_lo turns the low add into the
// subtraction, so the result is bit-identical to
//   acc.re = acc.re + (p.re v.re - p.im v.im);  acc.im = acc.im + (p.re v.im + p.im v.re)
// with 4 instructions instead of 8.
__device__ __forceinline__ void cmac_exact(v2f &acc, v2f p, v2f v) {
    v2f t1, t2;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t1) : "v"(p), "v"(v));  // (pr vr, pr vi)
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t2) : "v"(p), "v"(v));  // (pi vi, pi vr)
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(t1) : "v"(t1), "v"(t2));  // product
    asm("v_pk_add_f32 %0, %0, %1" : "+v"(acc) : "v"(t1));
}

template <bool STORE>
__global__ void __launch_bounds__(NT) k_pn_correlate(const float2 *__restrict__ buf, long long N,
                                                     const float2 *__restrict__ pn, int L,
                                                     float thres, long long nl, int nblk,
                                                     unsigned long long *__restrict__ best,
                                                     float *__restrict__ mag) {
    __shared__ float2 xs[TILE + JC];
    __shared__ float4 ps[JC / 2];  // the chunk's PN taps, two per float4 (broadcast reads)
    __shared__ int stop;
    const int t = threadIdx.x;
    const int ch = blockIdx.x / nblk;
    const long long i0 = (long long)(blockIdx.x % nblk) * TILE;
    const unsigned long long key0 = (unsigned long long)ch * nl + i0;
    const float2 *x = buf + (long long)ch * N;
    // lane l of wave w owns lags i0 + 256 w + l + 64 k: the four LDS reads of
    // one tap are constant offsets (0, 512, 1024, 1536 B) from one address
    const int lb = (t >> 6) * (64 * LPT) + (t & 63);

    v2f acc[LPT];
#pragma unroll
    for (int k = 0; k < LPT; ++k) acc[k] = (v2f){0.f, 0.f};

    for (int j0 = 0; j0 < L; j0 += JC) {
        const int jn = L - j0 < JC ? L - j0 : JC;
        __syncthreads();  // previous chunk's reads of xs / stop are done
        if (!STORE && t == 0) stop = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= key0;
        for (int e = t; e < TILE + jn - 1; e += NT) {
            const long long gi = i0 + j0 + e;
            xs[e] = gi < N ? x[gi] : float2{0.f, 0.f};
        }
        for (int e = t; e < JC / 2; e += NT) {
            const float2 a = 2 * e < jn ? pn[j0 + 2 * e] : float2{0.f, 0.f};
            const float2 b = 2 * e + 1 < jn ? pn[j0 + 2 * e + 1] : float2{0.f, 0.f};
            ps[e] = float4{a.x, a.y, b.x, b.y};
        }
        __syncthreads();
        if (!STORE && stop) return;  // an earlier (channel, lag) already reached thres
        const float2 *xl = xs + lb;
        const float2 *pj = reinterpret_cast<const float2 *>(ps);
        int j = 0;
        for (; j + 4 <= jn; j += 4) {  // 4 taps: 8 + 2 LDS reads off two addresses, 128 VALU
            const float4 p01 = ps[j / 2], p23 = ps[j / 2 + 1];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float2 p = u == 0   ? float2{p01.x, p01.y}
                                 : u == 1 ? float2{p01.z, p01.w}
                                 : u == 2 ? float2{p23.x, p23.y}
                                          : float2{p23.z, p23.w};
#pragma unroll
                for (int k = 0; k < LPT; ++k) {
                    const float2 v = xl[j + u + 64 * k];
                    cmac_exact(acc[k], __builtin_bit_cast(v2f, p), __builtin_bit_cast(v2f, v));
                }
            }
        }
        for (; j < jn; ++j) {
            const float2 p = pj[j];
#pragma unroll
            for (int k = 0; k < LPT; ++k) {
                const float2 v = xl[j + 64 * k];
                cmac_exact(acc[k], __builtin_bit_cast(v2f, p), __builtin_bit_cast(v2f, v));
            }
        }
    }
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
        const long long i = i0 + lb + 64 * k;
        if (i >= nl) continue;
        const double dr = acc[k].x, di = acc[k].y;
        const float m = (float)__builtin_sqrt(dr * dr + di * di) / (float)L;  // hypotf / L
        const unsigned long long key = (unsigned long long)ch * nl + i;
        if (STORE) mag[key] = m;
        if (m >= thres) atomicMin(best, key);
    }
}

// sym[s][ch][k] = seq_ch[s*(C+cp) + cp + k], seq_ch = buf1[ch][lag+L .. N) ++ buf2[ch][0 .. lag)
__global__ void __launch_bounds__(256) k_pn_extract(const float2 *__restrict__ buf1,
                                                    const float2 *__restrict__ buf2, int R,
                                                    long long N, int L, long long nl,
                                                    const long long *__restrict__ pos, int C, int cp,
                                                    long long total, float2 *__restrict__ sym) {
    const long long p = *pos;
    if (p < 0) return;  // no hit: nothing to extract
    const long long lag = p % nl, head = N - lag - L;
    // element e = (s R + ch) C + k: sample cp + k of symbol s on channel ch
    auto put = [&](long long e, int k, int ch, long long s) {
        const long long q = s * (C + cp) + cp + k;
        const long long base = (long long)ch * N;
        sym[e] = q < head ? buf1[base + lag + L + q] : buf2[base + q - head];
    };
    if (total < 0x80000000ll) {  // 32-bit index math (a frame is far below 2^31 elements)
        for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < (unsigned)total; e += gridDim.x * 256u) {
            const unsigned r = e / (unsigned)C, s = r / (unsigned)R;
            put(e, (int)(e - r * (unsigned)C), (int)(r - s * (unsigned)R), s);
        }
        return;
    }
    for (long long e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long r = e / C, s = r / R;
        put(e, (int)(e - r * C), (int)(r - s * R), s);
    }
}

}  // namespace pn

hipError_t launch_pn_correlate(const float2 *buf, int R, long long N, const float2 *pn, int L,
                               float thres, long long *pos, float *mag, hipStream_t s) {
    const long long nl = N - L + 1;
    hipError_t e = hipMemsetAsync(pos, 0xff, sizeof(long long), s);  // -1 = ULLONG_MAX: no hit
    if (e != hipSuccess || nl <= 0 || R == 0) return e;
    const long long nblk = (nl + pn::TILE - 1) / pn::TILE;
    if (nblk * R > 0x7fffffffll) return hipErrorInvalidValue;
    auto *best = reinterpret_cast<unsigned long long *>(pos);
    // packed exact MAC (the scalar form is bit-identical and 5 % slower)
    if (mag)
        hipLaunchKernelGGL((pn::k_pn_correlate<true>), dim3((unsigned)(nblk * R)), dim3(pn::NT), 0, s, buf,
                           N, pn, L, thres, nl, (int)nblk, best, mag);
    else
        hipLaunchKernelGGL((pn::k_pn_correlate<false>), dim3((unsigned)(nblk * R)), dim3(pn::NT), 0, s,
                           buf, N, pn, L, thres, nl, (int)nblk, best, mag);
    return hipGetLastError();
}

hipError_t launch_pn_extract(const float2 *buf1, const float2 *buf2, int R, long long N, int L,
                             const long long *pos, int C, int cp, int nsym, float2 *sym,
                             hipStream_t s) {
    const long long total = (long long)nsym * R * C;
    if (total == 0) return hipSuccess;
    long long grid = (total + 255) / 256;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(pn::k_pn_extract, dim3((unsigned)grid), dim3(256), 0, s, buf1, buf2, R, N, L,
                       N - L + 1, pos, C, cp, total, sym);
    return hipGetLastError();
}

}  // namespace ofdm
