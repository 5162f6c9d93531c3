// lsmrc_freq.hip -- LS channel estimation and MRC combining on
// frequency-domain symbols (FFT already applied).
//
// These are the north-star kernels of the reference's GPU path re-designed
// for CDNA4:
//   findHs (gpuLS.cu:158-182) + findDistSqrd (gpuLS.cu:185-209)
//     -> k_ls_freq: one lane per subcarrier, antenna loop in registers
//        (coalesced along subcarriers, no shared-memory tree, no race), the
//        |H|^2 sum kept in the reference's sequential antenna order
//        (cpuLS.hpp:211-228).
//   multiplyWithChannelConj + combineForMRC + shiftOneRow (gpuLS.cu:109-125,
//   212-259) -> k_mrc_freq: one pass, no materialised R x K product tensor,
//   16-byte loads of two adjacent bins per lane, the output rotation folded
//   into the store index.
#include "common.hpp"
#include "launch.hpp"

#include <stdlib.h>

namespace ofdm {

__global__ void __launch_bounds__(256) k_ls_freq(const float2 *__restrict__ Y, long long frame_stride,
                                                 int R, int C, const float2 *__restrict__ X,
                                                 float2 *__restrict__ Hc, long long hc_fstride,
                                                 int hc_ld, int hc_jofs, float *__restrict__ P,
                                                 long long p_fstride, int p_jofs) {
    const int K = C - 1;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const long long f = blockIdx.y;
    const float2 *Yf = Y + f * frame_stride;
    float2 *Hf = Hc + f * hc_fstride;
    float *Pf = P + f * p_fstride;
    if (j < K) {
        const float2 x = X[j];
        float p = 0.f;
        for (int r = 0; r < R; ++r) {
            const float2 h = ls_conj(Yf[(long long)r * C + j + 1], x);
            Hf[(long long)r * hc_ld + j + hc_jofs] = h;
            // findDistSqrd: Hsqrd = Hsqrd + re*re + im*im, rows in order
            p = (r == 0) ? (h.x * h.x) + (h.y * h.y) : p + (h.x * h.x) + (h.y * h.y);
        }
        Pf[j + p_jofs] = p;
    }
    if (hc_jofs == 1 && j == 0) {  // bin layout: DC slot of H is 0, of P is 1
        for (int r = 0; r < R; ++r) Hf[(long long)r * hc_ld] = float2{0.f, 0.f};
        if (p_jofs == 1) Pf[0] = 1.f;
    }
}

hipError_t launch_ls_freq(const float2 *Y, long long frame_stride, long long nframes, int R, int C,
                          const float2 *X, float2 *Hc, long long hc_fstride, int hc_ld, int hc_jofs,
                          float *P, long long p_fstride, int p_jofs, hipStream_t s) {
    if (nframes <= 0) return hipSuccess;
    const int K = C - 1;
    const long long maxy = 65535;
    for (long long f0 = 0; f0 < nframes; f0 += maxy) {
        const long long n = nframes - f0 < maxy ? nframes - f0 : maxy;
        hipLaunchKernelGGL(k_ls_freq, dim3((K + 255) / 256, (unsigned)n), dim3(256), 0, s,
                           Y + f0 * frame_stride, frame_stride, R, C, X, Hc + f0 * hc_fstride,
                           hc_fstride, hc_ld, hc_jofs, P + f0 * p_fstride, p_fstride, p_jofs);
    }
    return hipGetLastError();
}

// One lane = two adjacent bins (b = 2m, 2m+1) of one data symbol.
template <bool BIN_LAYOUT>
__global__ void __launch_bounds__(256) k_mrc_freq(const float2 *__restrict__ Y, long long frame_stride,
                                                  long long sym_stride, long long nq, int nsym, int R,
                                                  int C, const float2 *__restrict__ Hc,
                                                  long long hc_fstride, int hc_ld, int hc_jofs,
                                                  const float *__restrict__ P, long long p_fstride,
                                                  int p_jofs, float2 *__restrict__ out, int mode) {
    const int K = C - 1;
    const int pairs = C / 2;
    const int bps = (pairs + blockDim.x - 1) / blockDim.x;  // blocks per symbol
    const long long q = (long long)blockIdx.x / bps;
    const int m = (int)(blockIdx.x % bps) * blockDim.x + threadIdx.x;
    if (q >= nq || m >= pairs) return;
    const long long f = q / nsym;
    const long long sd = q % nsym;
    const float2 *Ys = Y + f * frame_stride + sd * sym_stride + 2 * m;
    const float2 *Hf = Hc + f * hc_fstride;
    const int j0 = 2 * m - 1, j1 = 2 * m;  // subcarriers of bins 2m, 2m+1
    float2 a0{0.f, 0.f}, a1{0.f, 0.f};
    for (int r = 0; r < R; ++r) {
        const float4 y = *reinterpret_cast<const float4 *>(Ys + (long long)r * C);
        float2 h0, h1;
        if (BIN_LAYOUT) {  // Hc(r, b) at r*hc_ld + b, DC slot zero
            const float4 h = *reinterpret_cast<const float4 *>(Hf + (long long)r * hc_ld + 2 * m);
            h0 = float2{h.x, h.y};
            h1 = float2{h.z, h.w};
        } else {
            const float2 *hr = Hf + (long long)r * hc_ld + hc_jofs;
            h0 = m > 0 ? hr[j0] : float2{0.f, 0.f};
            h1 = hr[j1];
        }
        // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
        a0.x = a0.x + (y.x * h0.x - y.y * h0.y);
        a0.y = a0.y + (y.x * h0.y + y.y * h0.x);
        a1.x = a1.x + (y.z * h1.x - y.w * h1.y);
        a1.y = a1.y + (y.z * h1.y + y.w * h1.x);
    }
    float2 *o = out + q * K;
    if (mode == 0) {
        const float *Pf = P + f * p_fstride + p_jofs;
        if (m > 0) {
            const float p0 = Pf[j0];
            o[out_pos(j0, K)] = float2{a0.x * __builtin_amdgcn_rcpf(p0), a0.y * __builtin_amdgcn_rcpf(p0)};
        }
        const float p1 = Pf[j1];
        o[out_pos(j1, K)] = float2{a1.x * __builtin_amdgcn_rcpf(p1), a1.y * __builtin_amdgcn_rcpf(p1)};
    } else {
        if (m > 0) o[j0] = a0;
        o[j1] = a1;
    }
}

// Odd C (no 16-byte bin pairs): one lane = one subcarrier j of one data
// symbol; Hc(r, j) at r*hc_ld + j + hofs (hofs = 1 in the bin layout).
__global__ void __launch_bounds__(256) k_mrc_freq1(const float2 *__restrict__ Y, long long frame_stride,
                                                   long long sym_stride, long long nq, int nsym, int R, int C,
                                                   const float2 *__restrict__ Hc, long long hc_fstride, int hc_ld,
                                                   int hofs, const float *__restrict__ P, long long p_fstride,
                                                   int p_jofs, float2 *__restrict__ out, int mode) {
    const int K = C - 1;
    const int bps = (K + blockDim.x - 1) / blockDim.x;
    const long long q = (long long)blockIdx.x / bps;
    const int j = (int)(blockIdx.x % bps) * blockDim.x + threadIdx.x;
    if (q >= nq || j >= K) return;
    const long long f = q / nsym;
    const float2 *Ys = Y + f * frame_stride + (q % nsym) * sym_stride + j + 1;
    const float2 *Hf = Hc + f * hc_fstride + j + hofs;
    float2 a{0.f, 0.f};
    for (int r = 0; r < R; ++r) {
        const float2 y = Ys[(long long)r * C], h = Hf[(long long)r * hc_ld];
        // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
        a.x = a.x + (y.x * h.x - y.y * h.y);
        a.y = a.y + (y.x * h.y + y.y * h.x);
    }
    if (mode == 0) {
        const float p = P[f * p_fstride + p_jofs + j];
        out[q * K + out_pos_any(j, K)] = float2{a.x * __builtin_amdgcn_rcpf(p), a.y * __builtin_amdgcn_rcpf(p)};
    } else {
        out[q * K + j] = a;
    }
}

// Bin-layout MRC over whole frames (ofdm_frame_demod_freq, the staged path):
// one lane = two adjacent bins of G consecutive data symbols of ONE frame,
// so each Hc float4 read from L2 serves G symbols, and the antenna loop is
// unrolled by U with all U (G + 1) 16-byte loads of a step issued before
// its MACs (U (G + 1) x 1 KiB in flight per wave).  Blocks are numbered
// (frame, symbol group, bin chunk), bin chunk fastest, and mapped so that a
// frame's blocks run on one XCD (its Hc rows stay in one L2).  Tail groups
// repeat the frame's last symbol without storing it.
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_load4(const float4 *p) {
    return __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p)));
}

template <int G, int U, bool NT = true>
__global__ void __launch_bounds__(256) k_mrc_freq_frames(const float2 *__restrict__ Y, long long frame_stride,
                                                         long long sym_stride, int nsym, int R, int C,
                                                         const float2 *__restrict__ Hc, long long hc_fstride,
                                                         const float *__restrict__ P, long long p_fstride,
                                                         int p_jofs, float2 *__restrict__ out, int mode,
                                                         long long nblocks, long long per_xcd, int bps) {
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);
    if (lb >= nblocks) return;
    const int K = C - 1;
    const int gpf = (nsym + G - 1) / G;
    const long long rest = lb / bps;
    const int m = (int)(lb - rest * bps) * blockDim.x + threadIdx.x;
    if (m >= C / 2) return;
    const long long f = rest / gpf;
    const int s0 = (int)(rest - f * gpf) * G;
    const float4 *Yq[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int sd = s0 + g < nsym ? s0 + g : nsym - 1;
        Yq[g] = reinterpret_cast<const float4 *>(Y + f * frame_stride + sd * sym_stride + 2 * m);
    }
    const float4 *Hq = reinterpret_cast<const float4 *>(Hc + f * hc_fstride + 2 * m);
    const int ld4 = C / 2;  // row pitch in float4
    float2 a0[G], a1[G];
#pragma unroll
    for (int g = 0; g < G; ++g) a0[g] = a1[g] = float2{0.f, 0.f};
    auto mac = [&](const float4 &h, const float4 (&y)[G]) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
            a0[g].x = a0[g].x + (y[g].x * h.x - y[g].y * h.y);
            a0[g].y = a0[g].y + (y[g].x * h.y + y[g].y * h.x);
            a1[g].x = a1[g].x + (y[g].z * h.z - y[g].w * h.w);
            a1[g].y = a1[g].y + (y[g].z * h.w + y[g].w * h.z);
        }
    };
    int r = 0;
    for (; r + U <= R; r += U) {
        float4 h[U], y[U][G];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            h[u] = Hq[(long long)(r + u) * ld4];
#pragma unroll
            for (int g = 0; g < G; ++g)
                y[u][g] = NT ? nt_load4(Yq[g] + (long long)(r + u) * ld4) : Yq[g][(long long)(r + u) * ld4];
        }
        __builtin_amdgcn_sched_barrier(0);  // all U (G + 1) loads in flight before the first MAC
#pragma unroll
        for (int u = 0; u < U; ++u) mac(h[u], y[u]);
    }
    for (; r < R; ++r) {
        float4 y[G];
        const float4 h = Hq[(long long)r * ld4];
#pragma unroll
        for (int g = 0; g < G; ++g) y[g] = NT ? nt_load4(Yq[g] + (long long)r * ld4) : Yq[g][(long long)r * ld4];
        mac(h, y);
    }
    const int j0 = 2 * m - 1, j1 = 2 * m;  // subcarriers of bins 2m, 2m+1
    // P is read only when dividing (mode 0): a numerator-only caller may pass none
    const float *Pf = P + f * p_fstride + p_jofs;
    const float p0 = (mode == 0 && m > 0) ? Pf[j0] : 1.f, p1 = mode == 0 ? Pf[j1] : 1.f;
    const int o0 = mode == 0 ? out_pos(j0 < 0 ? 0 : j0, K) : j0, o1 = mode == 0 ? out_pos(j1, K) : j1;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (s0 + g >= nsym) break;
        float2 *o = out + (f * nsym + s0 + g) * (long long)K;
        float2 v0 = a0[g], v1 = a1[g];
        if (mode == 0) {
            // one reciprocal and two products per bin (within 2 ulp of the
            // two divisions; frame_td.hip hlds_epilogue)
            const float r0 = __builtin_amdgcn_rcpf(p0), r1 = __builtin_amdgcn_rcpf(p1);
            v0 = float2{v0.x * r0, v0.y * r0};
            v1 = float2{v1.x * r1, v1.y * r1};
        }
        if (m > 0)
            __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, v0),
                                        reinterpret_cast<unsigned long long *>(o + o0));
        __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, v1),
                                    reinterpret_cast<unsigned long long *>(o + o1));
    }
}

hipError_t launch_mrc_freq(const float2 *Y, long long frame_stride, long long sym_stride,
                           long long nframes, int nsym, int R, int C, const float2 *Hc,
                           long long hc_fstride, int hc_ld, int hc_jofs, const float *P,
                           long long p_fstride, int p_jofs, float2 *out, int mode, hipStream_t s) {
    const long long nq = nframes * nsym;
    if (nq <= 0) return hipSuccess;
    if (C >= 512 && (C % 2) == 0 && hc_jofs == 0 && hc_ld == C && (hc_fstride % 2) == 0 &&
        (sym_stride % 2) == 0 &&
        (frame_stride % 2) == 0 && ((uintptr_t)Hc % 16) == 0 && ((uintptr_t)Y % 16) == 0) {
        const int bps = (C / 2 + 255) / 256;  // C = 1200, 1536, ...: a partial last chunk
        // same-process A/B (profiles/r2_ab/abf_*): 8 symbols per lane at C <= 2048
        // (2 waves/SIMD, 32 KiB in flight per wave), 4 at C = 4096
        auto kern = C >= 4096 ? k_mrc_freq_frames<4, 4> : k_mrc_freq_frames<8, 4>;
        int g = C >= 4096 ? 4 : 8;
        const long long nbg = nframes * ((nsym + g - 1) / g) * bps, pxg = (nbg + 7) / 8;
        if (pxg * 8 > 0x7fffffffll) return hipErrorInvalidValue;
        hipLaunchKernelGGL(kern, dim3((unsigned)(pxg * 8)), dim3(256), 0, s, Y, frame_stride, sym_stride, nsym, R,
                           C, Hc, hc_fstride, P, p_fstride, p_jofs, out, mode, nbg, pxg, bps);
        return hipGetLastError();
    }
    if (C & 1) {
        const int bps = (C - 1 + 255) / 256;
        const long long blocks = nq * bps;
        if (blocks > 0x7fffffffll) return hipErrorInvalidValue;
        const int hofs = (hc_jofs == 0 && hc_ld == C) ? 1 : hc_jofs;  // bin layout: subcarrier j at bin j + 1
        hipLaunchKernelGGL(k_mrc_freq1, dim3((unsigned)blocks), dim3(256), 0, s, Y, frame_stride, sym_stride, nq,
                           nsym, R, C, Hc, hc_fstride, hc_ld, hofs, P, p_fstride, p_jofs, out, mode);
        return hipGetLastError();
    }
    const int threads = C / 2 < 256 ? 64 * ((C / 2 + 63) / 64) : 256;
    const int bps = (C / 2 + threads - 1) / threads;
    const long long blocks = nq * bps;
    if (blocks > 0x7fffffffll) return hipErrorInvalidValue;
    const bool bin = (hc_jofs == 0 && hc_ld == C && (hc_fstride % 2) == 0 &&
                      ((uintptr_t)Hc % 16) == 0);
    if (bin)
        hipLaunchKernelGGL(k_mrc_freq<true>, dim3((unsigned)blocks), dim3(threads), 0, s, Y,
                           frame_stride, sym_stride, nq, nsym, R, C, Hc, hc_fstride, hc_ld, hc_jofs,
                           P, p_fstride, p_jofs, out, mode);
    else
        hipLaunchKernelGGL(k_mrc_freq<false>, dim3((unsigned)blocks), dim3(threads), 0, s, Y,
                           frame_stride, sym_stride, nq, nsym, R, C, Hc, hc_fstride, hc_ld, hc_jofs,
                           P, p_fstride, p_jofs, out, mode);
    return hipGetLastError();
}

// Element e = q K + j of [e0, e0 + count): out[q][out_pos(j)] = num / P[f][j].
// Grid-stride; the (symbol, subcarrier) pair is carried from one stride to
// the next and the frame formed by a 32-bit division, so that the loop holds
// none of the three 64-bit divisions per element it had (VALU-bound at
// 4.2 TB/s).
__global__ void __launch_bounds__(256) k_mrc_finalize(const float2 *__restrict__ num, long long e0,
                                                      long long count, int nsym, int K,
                                                      const float *__restrict__ P,
                                                      float2 *__restrict__ out) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    long long q = (e0 + i) / K;
    int j = (int)(e0 + i - q * K);
    const long long dq = stride / K;
    const int dj = (int)(stride - dq * K);
    for (; i < count; i += stride) {
        const long long f = q < 0x100000000ll ? (long long)((unsigned)q / (unsigned)nsym) : q / nsym;
        const float p = P[f * K + j];
        const float2 v = num[i];
        out[q * K + out_pos_any(j, K)] = float2{v.x * __builtin_amdgcn_rcpf(p), v.y * __builtin_amdgcn_rcpf(p)};
        q += dq;
        j += dj;
        if (j >= K) {
            j -= K;
            ++q;
        }
    }
}

hipError_t launch_mrc_finalize(const float2 *num, long long e0, long long count, int nsym, int K,
                               const float *P, float2 *out, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    long long blocks = (count + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_mrc_finalize, dim3((unsigned)blocks), dim3(256), 0, s, num, e0, count, nsym, K,
                       P, out);
    return hipGetLastError();
}

}  // namespace ofdm
