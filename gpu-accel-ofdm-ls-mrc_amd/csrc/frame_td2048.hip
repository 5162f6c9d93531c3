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

#include <stdlib.h>

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
template <bool NT>
__device__ __forceinline__ void row_fft2048(const float2 *__restrict__ src, int t, float2 *T,
                                            const float2 *lds, float2 (&xe)[16], float2 (&xo)[16]) {
    const float2 *tw1 = lds, *tw2 = lds + hl::TW1S, *twv = lds + hl::TW1S + hl::TW2S;
    float2 u[16], v[16];
    row_load<NT>(src, t, u);
    row_load<NT>(src + HALF, t, v);
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

// Same FFT with the row already in registers (lo = x[n], hi = x[n + 1024]),
// the DIF split done in place.  PREF: the next row is loaded into lo (hi) as
// soon as the first (second) half-FFT has written it to the transpose image,
// so it is in flight during the rest of this row.
// Each half is combined as soon as it is transformed (ae += X[2 b] Hc[2 b],
// ao += X[2 b + 1] Hc[2 b + 1], Hc row hr in LDS, float4 lane order), so only
// one half's bins are live at a time.
template <bool NOHC = false>
__device__ __forceinline__ void mac_half(const float2 *hr, int e, int t, const float2 (&x)[16],
                                         float2 (&acc)[16]) {
    // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        // NOHC: diagnostic only (wrong results), no Hc reads
        const float2 h = NOHC ? float2{1.f, (float)k} : hr[2 * (k * 64 + t) + e];
        acc[k].x = acc[k].x + (x[k].x * h.x - x[k].y * h.y);
        acc[k].y = acc[k].y + (x[k].x * h.y + x[k].y * h.x);
    }
}

// TWC: no W2048^n table in LDS; W2048^(t + 64 m) = W2048^t W32^m is formed
// from the lane's W2048^t (wt) and the wave-uniform W32^m (scalar loads).
template <bool NT, bool PREF, bool NOHC = false, bool TWC = false>
__device__ __forceinline__ void row_fft2048_pf(const float2 *__restrict__ next, int t, float2 *T,
                                               const float2 *lds, float2 (&lo)[16], float2 (&hi)[16],
                                               const float2 *hr, float2 (&ae)[16], float2 (&ao)[16],
                                               float2 wt = float2{1.f, 0.f}) {
    float2 x[16];
    const float2 *tw1 = lds, *tw2 = lds + hl::TW1S, *twv = lds + hl::TW1S + hl::TW2S;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const float2 d = csub(lo[m], hi[m]);
        lo[m] = cadd(lo[m], hi[m]);
        hi[m] = cmul(d, TWC ? cmul(wt, g_tw[64 * m * (OFDM_TW_N / C)]) : twv[m * 64 + t]);
    }
    hl::row_fft_a(lo, t, T, tw1);
    __builtin_amdgcn_sched_barrier(0);
    if (PREF) row_load<NT>(next, t, lo);
    hl::row_fft_b(t, T, tw2, x);
    mac_half<NOHC>(hr, 0, t, x, ae);
    hl::row_fft_a(hi, t, T, tw1);
    __builtin_amdgcn_sched_barrier(0);
    if (PREF) row_load<NT>(next + HALF, t, hi);
    hl::row_fft_b(t, T, tw2, x);
    mac_half<NOHC>(hr, 1, t, x, ao);
}

// ---------------------------------------------------------------------------
// LS: one workgroup (4 waves) per frame, wave w takes antenna rows w, w+4, ...
// Pilots (K values) in LDS; partial |H|^2 per wave combined in wave order.
// ---------------------------------------------------------------------------
constexpr int LS_WAVES = 4;
constexpr size_t LS_LDS = lds_bytes(LS_WAVES) + (size_t)C * sizeof(float2);

__global__ void __launch_bounds__(256) k_ls_td2048(const float2 *__restrict__ iq, int S, int R,
                                                   int prefix, const float2 *__restrict__ X,
                                                   float2 *__restrict__ Hc, float *__restrict__ P,
                                                   int partial) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float2 *T = lds + TAB + w * hl::TS;
    float2 *xs = lds + TAB + LS_WAVES * hl::TS;  // xs[b] = X[b - 1], xs[0] unused
    fill_tables(lds);
    for (int b = threadIdx.x; b < C; b += blockDim.x) xs[b] = b ? X[b - 1] : float2{1.f, 0.f};
    __syncthreads();

    const long long f = blockIdx.x;
    const int Cp = C + prefix;
    const float2 *pilot = iq + f * (long long)S * R * Cp + prefix;
    float4 *Hf = reinterpret_cast<float4 *>(Hc + f * (long long)R * C);
    const int b0 = lane_bin0(t);
    float pe[16], po[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) pe[k] = po[k] = 0.f;
    for (int r = w; r < R; r += LS_WAVES) {
        float2 xe[16], xo[16];
        row_fft2048<false>(pilot + (long long)r * Cp, t, T, lds, xe, xo);
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
        Pf[b] = b == 0 ? (partial ? 0.f : 1.f) : sum;
    }
}

// ---------------------------------------------------------------------------
// MRC: one wave per data symbol, MRC_WAVES consecutive symbols per workgroup,
// XCD-grouped block order (as k_mrc_td1024).  ~190 VGPRs -> 2 waves/SIMD.
// mode 0: out[q][out_pos(j)] = acc / P;  mode 1: out[q][j] = acc (numerator)
// ---------------------------------------------------------------------------
constexpr int MRC_WAVES = 4;

template <bool NT, int DBG = 0>
__global__ void __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(2, 2)))
k_mrc_td2048(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
             const float *__restrict__ P, float2 *__restrict__ out, long long nq, long long nblocks,
             long long per_xcd, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float2 *T = lds + TAB + w * hl::TS;
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);
    if (lb >= nblocks) return;
    fill_tables(lds);
    __syncthreads();
    const long long q = lb * MRC_WAVES + w;
    if (q >= nq) return;  // no block-level sync follows

    const int nsym = S - 1;
    const long long f = q / nsym;
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const float4 *Hf = reinterpret_cast<const float4 *>(Hc + f * (long long)R * C);

    float2 ae[16], ao[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) ae[k] = ao[k] = float2{0.f, 0.f};
    if constexpr ((DBG & 4) != 0) {
        // diagnostic only (wrong results): the row prefetch of k_mrc_td2048h
        // without any Hc reads -- bounds what a prefetching kernel could gain
        float2 lo[16], hi[16];
        row_load<NT>(sym, t, lo);
        row_load<NT>(sym + HALF, t, hi);
        for (int r = 0; r < R; ++r)
            row_fft2048_pf<NT, true, true>(sym + (long long)(r + 1 < R ? r + 1 : r) * Cp, t, T, lds, lo, hi,
                                           nullptr, ae, ao);
    }
    for (int r = 0; r < ((DBG & 4) ? 0 : R); ++r) {
        float2 xe[16], xo[16];
        row_fft2048<NT>(sym + (long long)r * Cp, t, T, lds, xe, xo);
        __builtin_amdgcn_sched_barrier(0);
        const float4 *hr = Hf + (long long)r * (C / 2);
        // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            // DBG & 2: diagnostic only (wrong results), no Hc traffic
            const float4 h = (DBG & 2) ? float4{1.f, (float)k, (float)k, 1.f} : hr[k * 64 + t];
            ae[k].x = ae[k].x + (xe[k].x * h.x - xe[k].y * h.y);
            ae[k].y = ae[k].y + (xe[k].x * h.y + xe[k].y * h.x);
            ao[k].x = ao[k].x + (xo[k].x * h.z - xo[k].y * h.w);
            ao[k].y = ao[k].y + (xo[k].x * h.w + xo[k].y * h.z);
        }
    }
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    if ((mode & 1) == 0) {
        const float *Pf = P + f * C;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            if (be > 0) {
                const float pv = Pf[be];
                o[out_pos(be - 1, K)] = float2{ae[k].x / pv, ae[k].y / pv};
            }
            const float pv = Pf[be + 1];
            o[out_pos(be, K)] = float2{ao[k].x / pv, ao[k].y / pv};
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            if (be > 0) o[be - 1] = ae[k];
            o[be] = ao[k];
        }
    }
}

// k_mrc_td2048 with fewer live registers (k_mrc_td2048_lr, OFDM_MRC2K_LR=1):
// each FFT half is combined right after it is transformed, with that half's
// Hc words read from L2 just then (row_fft2048_pf without its prefetch), so
// only one half's bins and Hc are live -- WPE = 3 waves per SIMD instead of 2
// (12 per CU, LDS 51 KiB per 4-wave workgroup), more waves to cover the L2
// latency of the per-symbol Hc row.
template <bool NT, int WPE>
__global__ void __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(WPE, WPE)))
k_mrc_td2048_lr(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
                const float *__restrict__ P, float2 *__restrict__ out, long long nq, long long nblocks,
                long long per_xcd, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float2 *T = lds + TAB + w * hl::TS;
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);
    if (lb >= nblocks) return;
    fill_tables(lds);
    __syncthreads();
    const long long q = lb * MRC_WAVES + w;
    if (q >= nq) return;  // no block-level sync follows
    const int nsym = S - 1;
    const long long f = q / nsym;
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const float2 *Hf = Hc + f * (long long)R * C;  // float4 lane order read as float2 pairs
    float2 ae[16], ao[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) ae[k] = ao[k] = float2{0.f, 0.f};
    for (int r = 0; r < R; ++r) {
        float2 lo[16], hi[16];
        row_load<NT>(sym + (long long)r * Cp, t, lo);
        row_load<NT>(sym + (long long)r * Cp + HALF, t, hi);
        row_fft2048_pf<NT, false>(nullptr, t, T, lds, lo, hi, Hf + (long long)r * C, ae, ao);
    }
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    if ((mode & 1) == 0) {
        const float *Pf = P + f * C;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            if (be > 0) {
                const float pv = Pf[be];
                o[out_pos(be - 1, K)] = float2{ae[k].x / pv, ae[k].y / pv};
            }
            const float pv = Pf[be + 1];
            o[out_pos(be, K)] = float2{ao[k].x / pv, ao[k].y / pv};
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            if (be > 0) o[be - 1] = ae[k];
            o[be] = ao[k];
        }
    }
}

// ---------------------------------------------------------------------------
// MRC with the channel rows shared through LDS (k_mrc_td2048h): 8 waves = 8
// consecutive data symbols of ONE frame per workgroup (frame-aligned map,
// bpf = ceil((S-1)/8); tail waves repeat the frame's last symbol without
// storing).  The frame's 16 KiB Hc row is LDS-DMA'd once per workgroup into a
// double buffer instead of loaded by every wave from L2 (k_mrc_td2048 without
// its Hc loads ran 9.5 % faster: OFDM_MRC2K_DEBUG=2).  One barrier per row:
// after it, row r's Hc is visible and everyone has finished row r-1, whose
// buffer then receives row r+1.  LDS 16 KiB tables + 8 transpose images +
// 2 x 16 KiB = 117.5 KiB: one workgroup (2 waves/SIMD, as k_mrc_td2048) per CU.
// ---------------------------------------------------------------------------
// HW = 4 (two workgroups per CU, each in its own lockstep) drops the 8 KiB
// W2048^n table (TWC) so that 2 x (8 + 4 x 8.5 + 32) KiB fit.
template <int HW>
struct HLay {
    static constexpr bool TWC = HW < 8;
    static constexpr int TABH = TWC ? hl::TW1S + hl::TW2S : TAB;
    static constexpr size_t LDS = (size_t)(TABH + HW * hl::TS + 2 * C) * sizeof(float2);
    static_assert(LDS * (8 / HW) <= 160 * 1024, "8 waves per CU");
};
constexpr int H_WAVES = 8;

template <int HW>
__device__ __forceinline__ void dma_hc_row(const float2 *g, unsigned lds) {  // 16 KiB, 64 HW threads
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const char *src = reinterpret_cast<const char *>(g) + w * 1024 + lane * 16;
#pragma unroll
    for (int j = 0; j < 16 / HW; ++j) td1024::dma16(src + j * HW * 1024, lds + j * HW * 1024 + w * 1024);
}

template <bool NT, bool PF, int HW = H_WAVES>
__global__ void __attribute__((amdgpu_flat_work_group_size(64 * HW, 64 * HW), amdgpu_waves_per_eu(2, 2)))
k_mrc_td2048h(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
              const float *__restrict__ P, float2 *__restrict__ out, long long nblocks, long long per_xcd,
              int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    using L = HLay<HW>;
    static_assert(PF || !L::TWC, "the table-free twiddles are in the prefetching row loop only");
    float2 *T = lds + L::TABH + w * hl::TS;
    float2 *HB = lds + L::TABH + HW * hl::TS;  // [2][C]: Hc rows in the float4 lane order
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);  // XCD-grouped: a frame's blocks share an L2
    if (lb >= nblocks) return;  // whole workgroup
    const int nsym = S - 1;
    const long long bpf = (nsym + HW - 1) / HW;
    const long long f = lb / bpf;
    const int j = (int)(lb - f * bpf) * HW + w;  // data symbol index within the frame
    const bool store = j < nsym;
    const int s = 1 + (store ? j : nsym - 1);
    const float2 *Hg = Hc + f * (long long)R * C;
    const unsigned hb[2] = {td1024::lds_addr(HB), td1024::lds_addr(HB + C)};
    dma_hc_row<HW>(Hg, hb[0]);  // row 0; landed at the first row's barrier
    if (L::TWC) hl::fill(lds, lds + hl::TW1S);
    else fill_tables(lds);
    __syncthreads();
    const float2 wt = g_tw[t * (OFDM_TW_N / C)];  // TWC: W2048^t

    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    float2 ae[16], ao[16], lo[16], hi[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) ae[k] = ao[k] = float2{0.f, 0.f};
    if (PF) {
        row_load<NT>(sym, t, lo);
        row_load<NT>(sym + HALF, t, hi);
    }
    for (int r = 0; r < R; ++r) {
        // row r's Hc (and, PF, its IQ) landed everywhere; everyone is done with row r-1's buffer
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (r + 1 < R) dma_hc_row<HW>(Hg + (long long)(r + 1) * C, hb[(r + 1) & 1]);
        if (PF) {
            const float2 *h2 = HB + (r & 1) * C;
            // the last row re-loads itself (one row in R) rather than branching:
            // two copies of the loop body would not fit the register budget
            row_fft2048_pf<NT, true, false, L::TWC>(sym + (long long)(r + 1 < R ? r + 1 : r) * Cp, t, T, lds,
                                                    lo, hi, h2, ae, ao, wt);
            continue;
        }
        float2 xe[16], xo[16];
        row_fft2048<NT>(sym + (long long)r * Cp, t, T, lds, xe, xo);
        __builtin_amdgcn_sched_barrier(0);
        const float4 *hr = reinterpret_cast<const float4 *>(HB + (r & 1) * C);
        // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const float4 h = hr[k * 64 + t];
            ae[k].x = ae[k].x + (xe[k].x * h.x - xe[k].y * h.y);
            ae[k].y = ae[k].y + (xe[k].x * h.y + xe[k].y * h.x);
            ao[k].x = ao[k].x + (xo[k].x * h.z - xo[k].y * h.w);
            ao[k].y = ao[k].y + (xo[k].x * h.w + xo[k].y * h.z);
        }
    }
    if (!store) return;
    const long long q = f * nsym + j;
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    if ((mode & 1) == 0) {
        const float *Pf = P + f * C;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            if (be > 0) {
                const float pv = Pf[be];
                o[out_pos(be - 1, K)] = float2{ae[k].x / pv, ae[k].y / pv};
            }
            const float pv = Pf[be + 1];
            o[out_pos(be, K)] = float2{ao[k].x / pv, ao[k].y / pv};
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 2 * (b0 + 16 * k);
            if (be > 0) o[be - 1] = ae[k];
            o[be] = ao[k];
        }
    }
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
                             const float2 *Hc, const float *P, float2 *out, int mode, hipStream_t s) {
    using namespace td2048;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    const long long nblocks = (nq + MRC_WAVES - 1) / MRC_WAVES;
    const long long per_xcd = (nblocks + 7) / 8;
    const long long grid = per_xcd * 8;
    if (grid > 0x7fffffffll) return hipErrorInvalidValue;
    // OFDM_MRC2K_H: k_mrc_td2048h, Hc rows shared through LDS.  1: 8 waves;
    // 2: 8 waves + the next IQ row prefetched; 4: 2 x 4 waves per CU + prefetch
    const char *hk = getenv("OFDM_MRC2K_H");
    const int hv = hk ? hk[0] - '0' : 0;
    if (hv == 1 || hv == 2 || hv == 4) {
        const int hw = hv == 4 ? 4 : H_WAVES;
        const long long bpf = ((S - 1) + hw - 1) / hw, nb = nframes * bpf, pxcd = (nb + 7) / 8;
        if (pxcd * 8 > 0x7fffffffll) return hipErrorInvalidValue;
        const void *kf = hv == 1   ? reinterpret_cast<const void *>(&k_mrc_td2048h<true, false>)
                         : hv == 2 ? reinterpret_cast<const void *>(&k_mrc_td2048h<true, true>)
                                   : reinterpret_cast<const void *>(&k_mrc_td2048h<true, true, 4>);
        const size_t lb = hv == 4 ? HLay<4>::LDS : HLay<H_WAVES>::LDS;
        if (hipError_t e = opt_in_lds(kf, (int)lb); e != hipSuccess) return e;  // > 64 KiB of dynamic LDS
        if (hv == 1)
            hipLaunchKernelGGL((k_mrc_td2048h<true, false>), dim3((unsigned)(pxcd * 8)), dim3(64 * hw), lb, s, iq,
                               S, R, prefix, Hc, P, out, nb, pxcd, mode);
        else if (hv == 2)
            hipLaunchKernelGGL((k_mrc_td2048h<true, true>), dim3((unsigned)(pxcd * 8)), dim3(64 * hw), lb, s, iq,
                               S, R, prefix, Hc, P, out, nb, pxcd, mode);
        else
            hipLaunchKernelGGL((k_mrc_td2048h<true, true, 4>), dim3((unsigned)(pxcd * 8)), dim3(64 * hw), lb, s,
                               iq, S, R, prefix, Hc, P, out, nb, pxcd, mode);
        return hipGetLastError();
    }
    const char *lr = getenv("OFDM_MRC2K_LR");  // 1: k_mrc_td2048_lr, 3 waves/SIMD; 2: same code, 2 waves/SIMD
    if (lr && (lr[0] == '1' || lr[0] == '2')) {
        if (lr[0] == '1')
            hipLaunchKernelGGL((k_mrc_td2048_lr<true, 3>), dim3((unsigned)grid), dim3(64 * MRC_WAVES),
                               lds_bytes(MRC_WAVES), s, iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd, mode);
        else
            hipLaunchKernelGGL((k_mrc_td2048_lr<true, 2>), dim3((unsigned)grid), dim3(64 * MRC_WAVES),
                               lds_bytes(MRC_WAVES), s, iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd, mode);
        return hipGetLastError();
    }
    if (getenv("OFDM_MRC2K_DEBUG") && getenv("OFDM_MRC2K_DEBUG")[0] == '6')
        hipLaunchKernelGGL((k_mrc_td2048<true, 6>), dim3((unsigned)grid), dim3(64 * MRC_WAVES),
                           lds_bytes(MRC_WAVES), s, iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd,
                           mode);
    else if (getenv("OFDM_MRC2K_DEBUG") && getenv("OFDM_MRC2K_DEBUG")[0] == '2')
        hipLaunchKernelGGL((k_mrc_td2048<true, 2>), dim3((unsigned)grid), dim3(64 * MRC_WAVES),
                           lds_bytes(MRC_WAVES), s, iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd,
                           mode);
    else if (getenv("OFDM_MRC_NTLOAD") && getenv("OFDM_MRC_NTLOAD")[0] == '0')
        hipLaunchKernelGGL((k_mrc_td2048<false>), dim3((unsigned)grid), dim3(64 * MRC_WAVES),
                           lds_bytes(MRC_WAVES), s, iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd,
                           mode);
    else
        hipLaunchKernelGGL((k_mrc_td2048<true>), dim3((unsigned)grid), dim3(64 * MRC_WAVES),
                           lds_bytes(MRC_WAVES), s, iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd,
                           mode);
    return hipGetLastError();
}

}  // namespace ofdm
