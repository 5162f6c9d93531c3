// frame_td.hip -- fused time-domain receiver for C = 1024 subcarriers.
//
// Replaces the reference's frame flow demodOneFrameCUDA (gpuLS.cu:575-675):
// batched cuFFT over all rows -> findHs -> findDistSqrd ->
// multiplyWithChannelConj -> combineForMRC -> shiftOneRow, six launches that
// each re-read the frame from global memory.  Here the time-domain IQ is read
// exactly once:
//
//   k_ls_td1024  one workgroup per frame: FFT the pilot rows (symbol 0),
//                Hc = conj(Y/X) stored bin-indexed [F][R][C], P = sum_r |Hc|^2.
//   k_mrc_td1024 one half-wave (32 lanes) per data symbol: for every antenna
//                row, a 1024-point FFT as 32 x 32 (in-register radix-2 32-point
//                FFTs, one LDS transpose), then acc += Y * Hc in registers;
//                finally acc / P stored at the rotated output position.
//
// 1024-point FFT on 32 lanes (four-step): lane l holds x[l + 32 m], m < 32.
//   A[l][k2] = FFT32_m(x[l + 32 m]) * W1024^(l k2)
//   X[k2 + 32 k1] = FFT32_l(A[l][k2])      (after an LDS transpose lane = k2)
// so lane l finally owns bins b = l + 32 k1, k1 < 32.
#include "common.hpp"
#include "launch.hpp"

namespace ofdm {
namespace td1024 {

constexpr int C = 1024;
constexpr int K = C - 1;
constexpr int TP = 33;            // padded pitch of 32x32 transposes (bank-conflict free)
constexpr int TBUF = 32 * TP;     // float2 per half-wave transpose region
constexpr int TWBUF = 32 * TP;    // block twiddle table W1024^(l*k2), [l][k2]

__device__ __forceinline__ void wave_lds_sync() {
    // LDS operations of one wave execute in order; this only stops the
    // compiler from moving LDS accesses across the exchange point.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void fill_twiddles(float2 *tw) {
    for (int i = threadIdx.x; i < TWBUF; i += blockDim.x) {
        const int l = i / TP, k2 = i % TP;
        tw[i] = k2 < 32 ? g_tw[((l * k2) & (C - 1)) * (OFDM_TW_N / C)] : float2{0.f, 0.f};
    }
}

// Forward 1024-point FFT of one row by the 32 lanes of a half-wave.
// src: first sample of the row (cyclic prefix already skipped).
// On return x[k1] = X[l + 32 k1].
__device__ __forceinline__ void row_fft(const float2 *__restrict__ src, int l, float2 *T,
                                        const float2 *tw, float2 (&x)[32]) {
    float2 a[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) a[m] = src[l + 32 * m];
    fft_reg<32, false>(a);
#pragma unroll
    for (int k2 = 1; k2 < 32; ++k2) a[k2] = cmul(a[k2], tw[l * TP + k2]);
#pragma unroll
    for (int k2 = 0; k2 < 32; ++k2) T[k2 * TP + l] = a[k2];
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = T[l * TP + i];
    wave_lds_sync();
    fft_reg<32, false>(x);
}

// ---------------------------------------------------------------------------
// LS: one workgroup (4 waves = 8 half-waves) per frame; half-wave h takes
// antenna rows h, h+8, ...; partial |H|^2 sums are combined in half-wave
// order through LDS (deterministic).
// partial != 0: antenna-split mode (P is a partial sum, DC slot 0).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ls_td1024(const float2 *__restrict__ iq, int S, int R,
                                                   int prefix, const float2 *__restrict__ X,
                                                   float2 *__restrict__ Hc, float *__restrict__ P,
                                                   int partial) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw = lds;
    const int half = threadIdx.x >> 5;  // 0..7
    const int l = threadIdx.x & 31;
    float2 *T = lds + TWBUF + half * TBUF;
    fill_twiddles(tw);
    __syncthreads();

    const long long f = blockIdx.x;
    const int Cp = C + prefix;
    const float2 *pilot = iq + f * (long long)S * R * Cp;
    float2 *Hf = Hc + f * (long long)R * C;
    float p[32];
#pragma unroll
    for (int k1 = 0; k1 < 32; ++k1) p[k1] = 0.f;
    // pilots of this lane's subcarriers: bin b = l + 32 k1 -> j = b - 1
    for (int r = half; r < R; r += 8) {
        float2 x[32];
        row_fft(pilot + (long long)r * Cp + prefix, l, T, tw, x);
        float2 *hr = Hf + (long long)r * C;
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) {
            const int b = l + 32 * k1;
            float2 h{0.f, 0.f};
            if (b > 0) h = ls_conj(x[k1], X[b - 1]);
            hr[b] = h;
            p[k1] = p[k1] + (h.x * h.x) + (h.y * h.y);
        }
    }
    __syncthreads();
    // partial sums -> LDS [half][bin] (reuses the transpose regions)
    float *pp = reinterpret_cast<float *>(lds + TWBUF);
#pragma unroll
    for (int k1 = 0; k1 < 32; ++k1) pp[half * C + l + 32 * k1] = p[k1];
    __syncthreads();
    float *Pf = P + f * C;
    for (int b = threadIdx.x; b < C; b += blockDim.x) {
        float s = pp[b];
        for (int h = 1; h < 8; ++h) s = s + pp[h * C + b];
        Pf[b] = b == 0 ? (partial ? 0.f : 1.f) : s;
    }
}

// ---------------------------------------------------------------------------
// MRC: workgroup = 4 waves = 8 half-waves = 8 consecutive data symbols.
// Workgroups are remapped so that consecutive symbols (which share a frame's
// Hc) land on the same XCD (blocks b and b+8 share an XCD under round-robin
// dispatch; speed only, never correctness).
// mode 0: out[q][out_pos(j)] = acc / P;  mode 1: out[q][j] = acc (numerator)
// ---------------------------------------------------------------------------
constexpr int MRC_WAVES = 4;
constexpr int MRC_SYMS = MRC_WAVES * 2;

__global__ void __launch_bounds__(256) k_mrc_td1024(const float2 *__restrict__ iq, int S, int R,
                                                    int prefix, const float2 *__restrict__ Hc,
                                                    const float *__restrict__ P,
                                                    float2 *__restrict__ out, long long nq,
                                                    long long nblocks, long long per_xcd, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw = lds;
    const int half = threadIdx.x >> 5;
    const int l = threadIdx.x & 31;
    float2 *T = lds + TWBUF + half * TBUF;
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);  // XCD-grouped logical block
    if (lb >= nblocks) return;
    fill_twiddles(tw);
    __syncthreads();

    long long q = lb * MRC_SYMS + half;
    const bool active = q < nq;
    if (!active) q = nq - 1;  // duplicate work, never stored
    const int nsym = S - 1;
    const long long f = q / nsym;
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const float2 *Hf = Hc + f * (long long)R * C;

    float2 acc[32];
#pragma unroll
    for (int k1 = 0; k1 < 32; ++k1) acc[k1] = float2{0.f, 0.f};
    for (int r = 0; r < R; ++r) {
        float2 x[32];
        row_fft(sym + (long long)r * Cp, l, T, tw, x);
        const float2 *hr = Hf + (long long)r * C + l;
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) {
            const float2 h = hr[32 * k1];
            acc[k1].x = acc[k1].x + (x[k1].x * h.x - x[k1].y * h.y);
            acc[k1].y = acc[k1].y + (x[k1].x * h.y + x[k1].y * h.x);
        }
    }
    if (!active) return;
    float2 *o = out + q * K;
    if (mode == 0) {
        const float *Pf = P + f * C;
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) {
            const int b = l + 32 * k1;
            if (b == 0) continue;
            const float pv = Pf[b];
            o[out_pos(b - 1, K)] = float2{acc[k1].x / pv, acc[k1].y / pv};
        }
    } else {
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) {
            const int b = l + 32 * k1;
            if (b > 0) o[b - 1] = acc[k1];
        }
    }
}

}  // namespace td1024

hipError_t launch_ls_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial, hipStream_t s) {
    using namespace td1024;
    if (nframes <= 0) return hipSuccess;
    const size_t lds = (TWBUF + 8 * TBUF) * sizeof(float2);
    hipLaunchKernelGGL(k_ls_td1024, dim3((unsigned)nframes), dim3(256), lds, s, iq, S, R, prefix, X, Hc,
                       P, partial);
    return hipGetLastError();
}

hipError_t launch_mrc_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode,
                             hipStream_t s) {
    using namespace td1024;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    const long long nblocks = (nq + MRC_SYMS - 1) / MRC_SYMS;
    const long long per_xcd = (nblocks + 7) / 8;
    const long long grid = per_xcd * 8;
    if (grid > 0x7fffffffll) return hipErrorInvalidValue;
    const size_t lds = (TWBUF + MRC_SYMS * TBUF) * sizeof(float2);
    hipLaunchKernelGGL(k_mrc_td1024, dim3((unsigned)grid), dim3(64 * MRC_WAVES), lds, s, iq, S, R,
                       prefix, Hc, P, out, nq, nblocks, per_xcd, mode);
    return hipGetLastError();
}

}  // namespace ofdm
