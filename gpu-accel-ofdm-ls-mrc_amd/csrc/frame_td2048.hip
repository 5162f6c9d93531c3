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
template <bool NT, bool LOAD = true, int PK = 0>
__device__ __forceinline__ void row_fft2048(const float2 *__restrict__ src, int t, float2 *T,
                                            const float2 *lds, float2 (&xe)[16], float2 (&xo)[16]) {
    const float2 *tw1 = lds, *tw2 = lds + hl::TW1S, *twv = lds + hl::TW1S + hl::TW2S;
    float2 u[16], v[16];
    if (LOAD) {
        row_load<NT>(src, t, u);
        row_load<NT>(src + HALF, t, v);
    } else {  // diagnostic: the previous row's spectrum stands in for the samples
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            u[m] = xe[m];
            v[m] = xo[m];
        }
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const float2 d = csub(u[m], v[m]);
        u[m] = cadd(u[m], v[m]);
        v[m] = cmul(d, twv[m * 64 + t]);
    }
    hl::row_fft_a<PK>(u, t, T, tw1);
    hl::row_fft_b<PK>(t, T, tw2, xe);
    hl::row_fft_a<PK>(v, t, T, tw1);
    hl::row_fft_b<PK>(t, T, tw2, xo);
}

// ---------------------------------------------------------------------------
// LS: one workgroup (4 waves) per frame, wave w takes antenna rows w, w+4, ...
// Pilots (K values) in LDS; partial |H|^2 per wave combined in wave order.
// ---------------------------------------------------------------------------
constexpr int LS_WAVES = 4;
constexpr size_t LS_LDS = lds_bytes(LS_WAVES) + (size_t)C * sizeof(float2);

// LS of frame f by a 4-wave workgroup.  WT (the one-launch kernel): Hc and P
// stored write-through (sc1) for the agent-scope hand-off.
template <bool WT>
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
            if constexpr (WT)
                td1024::store16_wt(Hf, R * C * 8, (r * (C / 2) + k * 64 + t) * 16, he, ho);
            else
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
        if constexpr (WT)
            td1024::store4_wt(Pf + b, v);
        else
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
    ls_frame2048<false>(iq, S, R, prefix, X, Hc, P, blockIdx.x, lds, w, t, partial);
}

// ---------------------------------------------------------------------------
// MRC: one wave per data symbol, MRC_WAVES consecutive symbols per workgroup,
// XCD-grouped block order (as k_mrc_td1024).  249 VGPRs (ILP scheduler) -> 2 waves/SIMD.
// mode 0: out[q][out_pos(j)] = acc / P;  mode 1: out[q][j] = acc (numerator)
// ---------------------------------------------------------------------------
constexpr int MRC_WAVES = 4;

// DBG (A/B build only): bit 1 no Hc loads, bit 2 no output stores (both
// wrong results by design), bit 3 the round-1 epilogue (scattered plain stores),
// bit 6 no IQ loads after the first row (compute only).
// PK: packed-f32 arithmetic (pk.hpp) -- bit 1 the first half of each
// 1024-point FFT (row_fft_a), bit 2 the second (row_fft_b), bit 4 the MAC.
// Default 6: 3-3.5 % faster than none under the ILP scheduler.
// IL = 1 (the default since round 3): the row's two FFT1024s
// software-pipelined through the transpose image as in k_mrc_td4096h
// (hlds::fa_* / fb_*, packed butterflies, recurrence twiddles, the MAC
// packed): A(u) -> write(u) -> read(u) -> A(v) while u's transpose is in
// flight -> write(v), read(v) -> the row's Hc loads -> B(u), B(v) -> MAC.
// Same-process A/B, R=64 x 200 frames: 4.06 vs 4.29 ms, outputs within
// 7.8e-7 of the round-2 row (profiles/r3/r3_ab_il_c2048.jsonl).  The next
// row's lower half issued after the DIF split (measured: 47 spilled VGPRs,
// 6.87 ms) was dropped.
template <int IL>
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
template <int DBG = 0, int PK = 6, int IL = 1>
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
    if constexpr (IL != 0) {
        const float2 *twv = lds + hl::TW1S + hl::TW2S;
        const hl::TwAnchors ca = hl::anchors_a(lds, t), cb = hl::anchors_b(lds + hl::TW1S, t);  // row invariants
        float2 lo[16];
        for (int r = 0; r < R; ++r)
            il_row<IL>(sym + (long long)r * Cp, Hf + (long long)r * (C / 2), t, T, twv, ca, cb, lo, ae, ao);
    }
    float2 xe[16], xo[16];
    for (int r = 0; r < (IL != 0 ? 0 : R); ++r) {
        if ((DBG & 64) && r > 0)
            row_fft2048<true, false>(sym, t, T, lds, xe, xo);
        else
            row_fft2048<true, true, PK>(sym + (long long)r * Cp, t, T, lds, xe, xo);
        __builtin_amdgcn_sched_barrier(0);
        const float4 *hr = Hf + (long long)r * (C / 2);
        // matrixMultThenSum (cpuLS.hpp:191-206): antennas summed in order.  With
        // PK & 4 (the default) the complex MAC is NOT the reference's
        // expression acc + (x.re h.re - x.im h.im): it is two FMA-contracted
        // packed steps (acc + x.re h) + (-x.im) h~, a reassociated sum that
        // matches cpuLS.hpp within the parity tolerance (1e-5), not bit for bit.
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const float4 h = (DBG & 2) ? float4{1.f, (float)k, (float)r, 1.f} : hr[k * 64 + t];
            if constexpr ((PK & 4) != 0) {  // packed MAC: (acc + x.re h) + (-x.im) h~, as k_mrc_td4096h
                pk::v2f a = pk::V(ae[k]), b = pk::V(ao[k]);
                pk::mac(a, pk::V(xe[k]), (pk::v2f){h.x, h.y});
                pk::mac(b, pk::V(xo[k]), (pk::v2f){h.z, h.w});
                ae[k] = pk::F(a);
                ao[k] = pk::F(b);
                continue;
            }
            ae[k].x = ae[k].x + (xe[k].x * h.x - xe[k].y * h.y);
            ae[k].y = ae[k].y + (xe[k].x * h.y + xe[k].y * h.x);
            ao[k].x = ao[k].x + (xo[k].x * h.z - xo[k].y * h.w);
            ao[k].y = ao[k].y + (xo[k].x * h.w + xo[k].y * h.z);
        }
    }
    if (DBG & 4) {  // diagnostic: no output stores (keep the sums live)
        float sacc = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) sacc += ae[k].x * ae[k].y + ao[k].x * ao[k].y;
        if (sacc == 1234.5f) out[q] = float2{sacc, 0.f};
        return;
    }
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    if (DBG & 8) {  // A/B: the round-1 epilogue, scattered plain stores
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
        return;
    }
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
            ae[k] = float2{ae[k].x / pv[k].x, ae[k].y / pv[k].x};
            ao[k] = float2{ao[k].x / pv[k].y, ao[k].y / pv[k].y};
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

template <int DBG = 0, int PK = 6, int IL = 1>
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
    mrc2048_symbol<DBG, PK, IL>(iq, S, R, prefix, Hc, P, out, q, t, T, lds, mode);

}

// One-launch frame demod (ofdm_frame_demod, C = 2048; frame_td.hip
// k_demod_td1024 for the protocol): workgroups 0 .. nls-1 estimate one frame
// each (write-through) and publish it; the MRC workgroups behind them wait
// for the (one or two) frames of their four symbols, or estimate them
// themselves when the bounded wait expires.  LDS: the LS layout (the MRC's
// plus the pilot row, whose first word carries the wait's outcome).
template <int DBG = 0>
__global__ void __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(2, 2)))
k_demod_td2048(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ X, float2 *Hc,
               float *P, float2 *__restrict__ out, long long nq, long long nblocks, long long per_xcd,
               unsigned long long *flags, unsigned long long epoch, int nls, long long nframes,
               long long spin_ticks) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    if ((int)blockIdx.x < nls) {  // estimator workgroup
        const long long f = blockIdx.x;
        if (f >= nframes) return;
        ls_frame2048<true>(iq, S, R, prefix, X, Hc, P, f, lds, w, t, 0);
        td1024::publish_flag(flags + f, epoch);
        return;
    }
    const long long pb = blockIdx.x - nls;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);
    if (lb >= nblocks) return;
    const int nsym = S - 1;
    const long long q0 = lb * MRC_WAVES, ql = q0 + MRC_WAVES - 1 < nq ? q0 + MRC_WAVES - 1 : nq - 1;
    int *seen = reinterpret_cast<int *>(lds + TAB + LS_WAVES * hl::TS);
    if (!td1024::consume_flags(flags, q0 / nsym, ql / nsym, epoch, spin_ticks, seen)) {
        for (long long ff = q0 / nsym; ff <= ql / nsym; ++ff)
            ls_frame2048<true>(iq, S, R, prefix, X, Hc, P, ff, lds, w, t, 0);
        td1024::acquire_all();
    }
    fill_tables(lds);
    __syncthreads();
    const long long q = q0 + w;
    if (q >= nq) return;
    mrc2048_symbol<DBG>(iq, S, R, prefix, Hc, P, out, q, t, lds + TAB + w * hl::TS, lds, 0);
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
    auto kern = k_mrc_td2048<0>;
#ifdef OFDM_AB_KNOBS
    if (ab_knob("MRC2K_IL", 1) == 0) kern = k_mrc_td2048<0, 6, 0>;  // round 2's row (FFTs one after the other)
    switch (ab_knob("MRC2K_DBG", 0)) {
        case 2: kern = k_mrc_td2048<2, 6, 0>; break;  // round-2 row
        case 4: kern = k_mrc_td2048<4, 6, 0>; break;  // round-2 row
        case 6: kern = k_mrc_td2048<6, 6, 0>; break;  // round-2 row
        case 8: kern = k_mrc_td2048<8, 6, 0>; break;  // round-2 row
        case 64: kern = k_mrc_td2048<64, 6, 0>; break;  // round-2 row
        default: break;
    }
    switch (ab_knob("MRC2K_PK", -1)) {  // packed-f32 parts other than the default 6
        case 0: kern = k_mrc_td2048<0, 0, 0>; break;
        case 1: kern = k_mrc_td2048<0, 1, 0>; break;
        case 2: kern = k_mrc_td2048<0, 2, 0>; break;
        case 3: kern = k_mrc_td2048<0, 3, 0>; break;
        case 7: kern = k_mrc_td2048<0, 7, 0>; break;
        default: break;
    }
#endif
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * MRC_WAVES), lds_bytes(MRC_WAVES), s, iq, S,
                       R, prefix, Hc, P, out, nq, nblocks, per_xcd, mode);
    return hipGetLastError();
}

#ifdef OFDM_AB_KNOBS  // A/B build only: no faster than the two launches
hipError_t launch_demod_td2048(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *X,
                               float2 *Hc, float *P, float2 *out, unsigned long long *flags,
                               unsigned long long epoch, hipStream_t s) {
    using namespace td2048;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    const long long nblocks = (nq + MRC_WAVES - 1) / MRC_WAVES;
    const long long per_xcd = (nblocks + 7) / 8;
    const long long nls = (nframes + 7) / 8 * 8;
    if (per_xcd * 8 + nls > 0x7fffffffll) return hipErrorInvalidValue;
    auto kern = k_demod_td2048<0>;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)LS_LDS); e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)(nls + per_xcd * 8)), dim3(64 * MRC_WAVES), LS_LDS, s, iq, S, R,
                       prefix, X, Hc, P, out, nq, nblocks, per_xcd, flags, epoch, (int)nls, nframes,
                       (long long)ab_knob("DEMOD_SPIN", (int)td1024::SPIN_TICKS));
    return hipGetLastError();
}
#endif

}  // namespace ofdm
