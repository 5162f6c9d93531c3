// frame_td2048.hip -- fused time-domain receiver for C = 2048 subcarriers
// (BASELINE configs[2]: 2048 subcarriers x 64 antennas).
//
// Same flow as frame_td.hip (one HBM pass over the IQ: demodOneFrameCUDA,
// gpuLS.cu:575-675, without its six re-reads), with a 2048-point FFT on one
// 64-lane wave built from the 1024-point wave FFT (wave_fft1024.hpp) by one
// decimation-in-frequency step done in registers:
//   lane t loads x[t + 64 m] and x[1024 + t + 64 m], m < 16;
//   u[n] = x[n] + x[n + 1024]               -> FFT1024 -> X[2 k]
//   v[n] = (x[n] - x[n + 1024]) W2048^n     -> FFT1024 -> X[2 k + 1]
// so lane (q, a) owns the bin pairs (2 b, 2 b + 1), b = b0(t) + 16 k.
//
// Hc "lane order" for C = 2048: per (frame, antenna) 1024 float4, float4
// k*64 + t = (Hc[2 b], Hc[2 b + 1]) of lane t's k-th pair -- 16 coalesced
// dwordx4 wave loads per row.  P stays bin-indexed [F][C].
#include "launch.hpp"
#include "wave_fft1024.hpp"
#include "diag.hpp"

OFDM_DIAG_TU(td2048)

namespace ofdm {
namespace td2048 {

using td1024::lane_bin0;
using td1024::row_load;
namespace hl = td1024::hlds;

constexpr int C = 2048;
constexpr int K = C - 1;
constexpr int HALF = 1024;
constexpr int TWV = 16 * 64;  // W2048^(t + 64 m), [m][t]
// LDS: TW1s | TW2s | TWV | per-wave transpose images
constexpr int TAB = hl::TW1S + hl::TW2S + TWV;
constexpr size_t lds_bytes(int waves) { return (size_t)(TAB + waves * hl::TS) * sizeof(float2); }

__device__ __forceinline__ void fill_tables(float2 *lds) {
    hl::fill(lds, lds + hl::TW1S);
    float2 *twv = lds + hl::TW1S + hl::TW2S;
    for (int i = threadIdx.x; i < TWV; i += blockDim.x) {
        const int m = i / 64, t = i % 64;
        twv[i] = g_tw[(t + 64 * m) * (OFDM_TW_N / C)];
    }
}

// FFT of one 2048-sample row (src) -> xe[k] = X[2 b], xo[k] = X[2 b + 1]
__device__ __forceinline__ void row_fft2048(const float2 *__restrict__ src, int t, float2 *T,
                                            const float2 *lds, float2 (&xe)[16], float2 (&xo)[16]) {
    const float2 *tw1 = lds, *tw2 = lds + hl::TW1S, *twv = lds + hl::TW1S + hl::TW2S;
    float2 u[16], v[16];
    row_load<false>(src, t, u);
    row_load<false>(src + HALF, t, v);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const float2 d = csub(u[m], v[m]);
        u[m] = cadd(u[m], v[m]);
        v[m] = cmul(d, twv[m * 64 + t]);
    }
    hl::row_fft_a(u, t, T, tw1);
    hl::row_fft_b(t, T, tw2, xe);
    hl::row_fft_a(v, t, T, tw1);
    hl::row_fft_b(t, T, tw2, xo);
}

// ---------------------------------------------------------------------------
// LS: one workgroup (4 waves) per frame, wave w takes antenna rows w, w+4, ...
// Pilots (K values) in LDS; partial |H|^2 per wave combined in wave order.
// ---------------------------------------------------------------------------
constexpr int LS_WAVES = 4;
constexpr size_t LS_LDS = lds_bytes(LS_WAVES) + (size_t)C * sizeof(float2);

// LS of frame f by a 4-wave workgroup.
__device__ __forceinline__ void ls_frame2048(const float2 *__restrict__ iq, int S, int R, int prefix,
                                             const float2 *__restrict__ X, float2 *Hc, float *P, long long f,
                                             float2 *lds, int w, int t, int partial) {
    float2 *T = lds + TAB + w * hl::TS;
    float2 *xs = lds + TAB + LS_WAVES * hl::TS;  // xs[b] = X[b - 1], xs[0] unused
    fill_tables(lds);
    for (int b = threadIdx.x; b < C; b += blockDim.x) xs[b] = b ? X[b - 1] : float2{1.f, 0.f};
    __syncthreads();

    const int Cp = C + prefix;
    const float2 *pilot = iq + f * (long long)S * R * Cp + prefix;
    float4 *Hf = reinterpret_cast<float4 *>(Hc + f * (long long)R * C);
    const int b0 = lane_bin0(t);
    float pe[16], po[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) pe[k] = po[k] = 0.f;
    for (int r = w; r < R; r += LS_WAVES) {
        float2 xe[16], xo[16];
        row_fft2048(pilot + (long long)r * Cp, t, T, lds, xe, xo);
        float4 *hr = Hf + (long long)r * (C / 2);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            // divideOneRow + conj (cpuLS.hpp:233-244, 303-307); DC bin dropped
            float2 he = ls_conj(xe[k], xs[be]);
            if (be == 0) he = float2{0.f, 0.f};
            const float2 ho = ls_conj(xo[k], xs[be + 1]);
            pe[k] = pe[k] + (he.x * he.x) + (he.y * he.y);  // findDistSqrd order
            po[k] = po[k] + (ho.x * ho.x) + (ho.y * ho.y);
            hr[k * 64 + t] = float4{he.x, he.y, ho.x, ho.y};
        }
    }
    __syncthreads();
    float *pp = reinterpret_cast<float *>(lds + TAB);  // [LS_WAVES][C], reuses T
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int be = 2 * (b0 + 16 * k);
        pp[w * C + be] = pe[k];
        pp[w * C + be + 1] = po[k];
    }
    __syncthreads();
    float *Pf = P + f * C;
    for (int b = threadIdx.x; b < C; b += blockDim.x) {
        float sum = pp[b];
        for (int i = 1; i < LS_WAVES; ++i) sum = sum + pp[i * C + b];  // antennas in order
        const float v = b == 0 ? (partial ? 0.f : 1.f) : sum;
        Pf[b] = v;
    }
    __syncthreads();  // pp (the transpose images) read before they are reused
}

__global__ void __launch_bounds__(256) k_ls_td2048(const float2 *__restrict__ iq, int S, int R,
                                                   int prefix, const float2 *__restrict__ X,
                                                   float2 *__restrict__ Hc, float *__restrict__ P,
                                                   int partial) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    ls_frame2048(iq, S, R, prefix, X, Hc, P, blockIdx.x, lds, w, t, partial);
}

// ---------------------------------------------------------------------------
// MRC: one wave per data symbol, MRC_WAVES consecutive symbols per workgroup,
// XCD-grouped block order (as k_mrc_td1024).  249 VGPRs (ILP scheduler) -> 2 waves/SIMD.
// mode 0: out[q][out_pos(j)] = acc / P;  mode 1: out[q][j] = acc (numerator)
// ---------------------------------------------------------------------------
constexpr int MRC_WAVES = 4;

// The row (since round 3): the row's two FFT1024s
// software-pipelined through the transpose image as in k_mrc_td4096h
// (hlds::fa_* / fb_*, packed butterflies, recurrence twiddles, the MAC
// packed): A(u) -> write(u) -> read(u) -> A(v) while u's transpose is in
// flight -> write(v), read(v) -> the row's Hc loads -> B(u), B(v) -> MAC.
// Same-process A/B, R=64 x 200 frames: 4.06 vs 4.29 ms, outputs within
// 7.8e-7 of the round-2 row (profiles/r3/r3_ab_il_c2048.jsonl).  The next
// row's lower half issued after the DIF split (measured: 47 spilled VGPRs,
// 6.87 ms) was dropped.
__device__ __forceinline__ void il_row(const float2 *__restrict__ src, const float4 *__restrict__ hr, int t, float2 *T, const float2 *twv,
                                       const hl::TwAnchors &ca, const hl::TwAnchors &cb, float2 (&lo)[16], float2 (&ae)[16],
                                       float2 (&ao)[16]) {
    using namespace pk;
    float2 hi[16];
    row_load<true>(src, t, lo);
    row_load<true>(src + HALF, t, hi);
    v2f u[16], v[16], xu[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const v2f d = sub(V(lo[m]), V(hi[m]));
        u[m] = add(V(lo[m]), V(hi[m]));
        v[m] = cmul(d, V(twv[m * 64 + t]));
    }
    hl::fa_compute(u, ca);
    hl::fa_write(u, t, T);
    hl::fb_read(t, T, xu);
    hl::fa_compute(v, ca);
    hl::fa_write(v, t, T);
    hl::fb_read(t, T, u);
    __builtin_amdgcn_sched_barrier(0);
    float4 h[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) h[k] = hr[k * 64 + t];
    __builtin_amdgcn_sched_barrier(0);
    float2 x[16];
    hl::fb_compute(xu, cb, t, x);
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // matrixMultThenSum (cpuLS.hpp:191-206), packed as the default kernel
        v2f a0 = V(ae[k]);
        pk::mac(a0, V(x[k]), (v2f){h[k].x, h[k].y});
        ae[k] = F(a0);
    }
    hl::fb_compute(u, cb, t, x);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        v2f a0 = V(ao[k]);
        pk::mac(a0, V(x[k]), (v2f){h[k].z, h[k].w});
        ao[k] = F(a0);
    }
}

// The MRC of data symbol q (< nq) by wave w (twiddle tables filled): rows,
// normalise (mode 0), rotated and staged stores.
__device__ __forceinline__ void mrc2048_symbol(const float2 *__restrict__ iq, int S, int R, int prefix,
                                               const float2 *Hc, const float *P, float2 *__restrict__ out,
                                               long long q, int t, float2 *T, float2 *lds, int mode) {
    const int nsym = S - 1;
    const long long f = q / nsym;
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const float4 *Hf = reinterpret_cast<const float4 *>(Hc + f * (long long)R * C);

    float2 ae[16], ao[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) ae[k] = ao[k] = float2{0.f, 0.f};
    const float2 *twv = lds + hl::TW1S + hl::TW2S;
    const hl::TwAnchors ca = hl::anchors_a(lds, t), cb = hl::anchors_b(lds + hl::TW1S, t);  // row invariants
    float2 lo[16];
    for (int r = 0; r < R; ++r)
        il_row(sym + (long long)r * Cp, Hf + (long long)r * (C / 2), t, T, twv, ca, cb, lo, ae, ao);
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    // normalise, then stage the 2047 outputs through this wave's transpose
    // image in two halves of 1024 positions and store each half as 16
    // contiguous 512-B nontemporal wave stores (instead of 32 scattered ones)
    if ((mode & 1) == 0) {
        const float *Pf = P + f * C;
        // all 16 |H|^2 pairs in flight before the first divide (left to
        // itself the compiler issues each load just before its use, behind a
        // vmcnt(0) wait: 16 serial L2 round trips per symbol)
        float2 pv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            pv[k] = *reinterpret_cast<const float2 *>(Pf + be);  // Pf[0] = 1: the DC slot
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            // one reciprocal (v_rcp_f32) and two products per bin instead of
            // two IEEE divisions (within 2 ulp; frame_td.hip hlds_epilogue)
            const float re = __builtin_amdgcn_rcpf(pv[k].x), ro = __builtin_amdgcn_rcpf(pv[k].y);
            ae[k] = float2{ae[k].x * re, ae[k].y * re};
            ao[k] = float2{ao[k].x * ro, ao[k].y * ro};
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            const int je = (mode & 1) ? be - 1 : out_pos(be - 1, K);  // be = 0: the DC bin, no output
            const int jo = (mode & 1) ? be : out_pos(be, K);
            if (be > 0 && (je >> 10) == h) T[((je & 1023) >> 6) * hl::TP + (je & 63)] = ae[k];
            if ((jo >> 10) == h) T[((jo & 1023) >> 6) * hl::TP + (jo & 63)] = ao[k];
        }
        td1024::wave_lds_sync();
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const int j = 1024 * h + t + 64 * m;
            if (j < K)
                __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, T[m * hl::TP + t]),
                                            reinterpret_cast<unsigned long long *>(o + j));
        }
        td1024::wave_lds_sync();
    }
}

__global__ void __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(2, 2)))
k_mrc_td2048(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
             const float *__restrict__ P, float2 *__restrict__ out, long long nq, long long nblocks,
             Tickets tk, long long k0, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float2 *T = lds + TAB + w * hl::TS;
    OFDM_DIAG_BEGIN()
    // the logical block (4 consecutive data symbols) is a work ticket
    // (wave_fft1024.hpp take_block); the slot is wave 0's transpose image,
    // first written after the table barrier
    const long long lb = td1024::wg_take_block(tk, nblocks, k0, blockIdx.x,
                                               reinterpret_cast<long long *>(lds + TAB));
    if (lb < 0) return;
    fill_tables(lds);
    __syncthreads();
    const long long q = lb * MRC_WAVES + w;
    if (q < nq) mrc2048_symbol(iq, S, R, prefix, Hc, P, out, q, t, T, lds, mode);  // no block-level sync inside
    OFDM_DIAG_END(td2048);

}

}  // namespace td2048

hipError_t launch_ls_td2048(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial, hipStream_t s) {
    using namespace td2048;
    if (nframes <= 0) return hipSuccess;
    if (nframes > 0x7fffffffll) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ls_td2048, dim3((unsigned)nframes), dim3(64 * LS_WAVES), LS_LDS, s, iq, S, R,
                       prefix, X, Hc, P, partial);
    return hipGetLastError();
}

hipError_t launch_mrc_td2048(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode, Tickets tk,
                             hipStream_t s) {
    using namespace td2048;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    const long long nblocks = (nq + MRC_WAVES - 1) / MRC_WAVES;
    const long long grid = td1024::ticket_grid(nblocks);
    if (grid > 0x7fffffffll) return hipErrorInvalidValue;
    auto kern = k_mrc_td2048;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * MRC_WAVES), lds_bytes(MRC_WAVES), s, iq, S,
                       R, prefix, Hc, P, out, nq, nblocks, tk, td1024::ticket_k0(2), mode);
    return hipGetLastError();
}


}  // namespace ofdm
