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
//   k_mrc_td1024 one wave (64 lanes) per data symbol: for every antenna row a
//                1024-point FFT in registers + one LDS transpose, then
//                acc += Y * Hc in registers (next row and its Hc prefetched);
//                finally acc / P stored at the rotated output position.
//
// 1024-point FFT on one wave (four-step, N = 64 x 16): lane t holds
// x[t + 64 m], m < 16.
//   A[t][k2]  = FFT16_m(x[t + 64 m]) * W1024^(t k2)                 k2 < 16
//   X[k2 + 16 k1] = DFT64_t(A[t][k2])                                k1 < 64
// The 64-point DFTs run on lane quads after an LDS transpose: lane
// t = 4 q + a (q = k2, a < 4) holds A[a + 4 l'][q], l' < 16, and
//   B_a[k'] = FFT16_l'(A[a + 4 l'][q]) * W64^(a k')                   k' < 16
//   X[q + 16 (k' + 16 c)] = sum_a B_a[k'] W4^(a c)                    c < 4
// the last sum being a radix-2 x 2 exchange inside the quad (DPP).  Lane
// (q, a) finally owns bins b = q + 256 c(a) + 16 k', c(a) = (a >> 1) + 2 (a & 1).
#include "launch.hpp"
#include "wave_fft1024.hpp"

#include <stdlib.h>

#include <type_traits>

namespace ofdm {
namespace td1024 {

// ---------------------------------------------------------------------------
// LS: one workgroup (4 waves) per frame; wave w takes antenna rows w, w+4, ...
// and keeps a partial |H|^2 per bin; partials are added in wave order through
// LDS (deterministic).  partial != 0: antenna-split mode (DC slot of P = 0).
// P is written bin-indexed [F][C]; Hc lane-ordered [F][R][8][64] float4.
// ---------------------------------------------------------------------------
constexpr int LS_WAVES = 4;

__global__ void __launch_bounds__(256) k_ls_td1024(const float2 *__restrict__ iq, int S, int R,
                                                   int prefix, const float2 *__restrict__ X,
                                                   float2 *__restrict__ Hc, float *__restrict__ P,
                                                   int partial) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw = lds;
    const int w = threadIdx.x >> 6;
    const int t = threadIdx.x & 63;
    float2 *T = lds + TWBUF + w * TBUF;
    fill_twiddles(tw);
    __syncthreads();

    const long long f = blockIdx.x;
    const int Cp = C + prefix;
    const float2 *pilot = iq + f * (long long)S * R * Cp + prefix;
    float4 *Hf = reinterpret_cast<float4 *>(Hc + f * (long long)R * C);
    const int b0 = lane_bin0(t);
    float2 xp[16];  // rotated pilots of this lane's subcarriers
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int b = b0 + 16 * k;
        xp[k] = b > 0 ? X[b - 1] : float2{1.f, 0.f};
    }
    float p[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) p[k] = 0.f;
    for (int r = w; r < R; r += LS_WAVES) {
        float2 a[16], x[16];
        row_load(pilot + (long long)r * Cp, t, a);
        row_fft(a, t, T, tw, x);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            float2 h = ls_conj(x[k], xp[k]);
            if (b0 + 16 * k == 0) h = float2{0.f, 0.f};
            x[k] = h;
            p[k] = p[k] + (h.x * h.x) + (h.y * h.y);
        }
        hc_store(Hf + (long long)r * (C / 2), t, x);
    }
    __syncthreads();
    float *pp = reinterpret_cast<float *>(lds + TWBUF);  // [LS_WAVES][C], reuses T
#pragma unroll
    for (int k = 0; k < 16; ++k) pp[w * C + b0 + 16 * k] = p[k];
    __syncthreads();
    float *Pf = P + f * C;
    for (int b = threadIdx.x; b < C; b += blockDim.x) {
        float sum = pp[b];
        for (int i = 1; i < LS_WAVES; ++i) sum = sum + pp[i * C + b];
        Pf[b] = b == 0 ? (partial ? 0.f : 1.f) : sum;
    }
}

// ---------------------------------------------------------------------------
// MRC: workgroup = WAVES waves = WAVES consecutive data symbols, one per wave.
// Workgroups are remapped so that consecutive symbols (which share a frame's
// Hc) land on the same XCD (blocks b and b+8 share an XCD under round-robin
// dispatch; speed only, never correctness).
// mode 0: out[q][out_pos(j)] = acc / P;  mode 1: out[q][j] = acc (numerator)
// Row-loop schedules (A/B-selectable at run time, OFDM_MRC_SCHED):
//   0 PREFETCH_COPY  next row loaded into a second buffer, copied at the top
//   1 NOPREFETCH     load, then compute (latency hidden by other waves)
// ---------------------------------------------------------------------------
enum { PREFETCH_COPY = 0, NOPREFETCH = 1 };

template <bool NT, int DBG = 0>
__device__ __forceinline__ void mrc_row(float2 (&a)[16], int t, float2 *T, const float2 *tw,
                                        const float4 *__restrict__ hr, float2 (&acc)[16]) {
    float2 h[16], x[16];
    if (DBG & 1) {  // diagnostic only: same memory traffic, no FFT
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = a[k];
    } else {
        row_fft(a, t, T, tw, x);
    }
    // keep the Hc loads (L2 hits) out of the FFT's register peak
    __builtin_amdgcn_sched_barrier(0);
    if (DBG & 2) {  // diagnostic only: no Hc traffic
#pragma unroll
        for (int k = 0; k < 16; ++k) h[k] = float2{1.f, (float)k};
    } else {
        hc_load(hr, t, h);
    }
    // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        acc[k].x = acc[k].x + (x[k].x * h[k].x - x[k].y * h[k].y);
        acc[k].y = acc[k].y + (x[k].x * h[k].y + x[k].y * h[k].x);
    }
}

// One symbol per wave.  PERSIST: a grid of ~2 workgroups per CU walks the
// symbol groups; each XCD (blocks b with equal b % 8 under round-robin
// dispatch; speed only) takes a contiguous range of groups so the frames in
// flight on an XCD share their Hc in its L2.
template <bool NT, int SCHED, int DBG, bool SYNC = false>
__device__ __forceinline__ void mrc_symbol(const float2 *__restrict__ iq, int S, int R, int prefix,
                                           const float2 *__restrict__ Hc, const float *__restrict__ P,
                                           float2 *__restrict__ out, long long q, int mode, int t,
                                           float2 *T, const float2 *tw, bool store = true) {
    const int nsym = S - 1;
    const long long f = q / nsym;
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const float4 *Hf = reinterpret_cast<const float4 *>(Hc + f * (long long)R * C);

    float2 acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = float2{0.f, 0.f};
    if (SCHED == PREFETCH_COPY) {
        float2 nxt[16];
        row_load<NT>(sym, t, nxt);
        for (int r = 0; r < R; ++r) {
            float2 a[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) a[m] = nxt[m];
            if (r + 1 < R) row_load<NT>(sym + (long long)(r + 1) * Cp, t, nxt);
            mrc_row<NT, DBG>(a, t, T, tw, Hf + (long long)r * (C / 2), acc);
        }
    } else {
        for (int r = 0; r < R; ++r) {
            float2 a[16];
            row_load<NT>(sym + (long long)r * Cp, t, a);
            // SYNC: the workgroup's waves (consecutive symbols, mostly one
            // frame) stay on the same antenna row, so its Hc row is fetched
            // from L2 once and re-read from L1
            if (SYNC) __syncthreads();
            mrc_row<NT, DBG>(a, t, T, tw, Hf + (long long)r * (C / 2), acc);
        }
    }
    if (!store) return;
    if (DBG & 4) {  // diagnostic only: no output stores
        float sacc = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) sacc += acc[k].x;
        if (sacc == 1234.5f) out[q] = float2{sacc, 0.f};
        return;
    }
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    if ((mode & 1) == 0) {
        const float *Pf = P + f * C + b0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int b = b0 + 16 * k;
            if (b == 0) continue;
            const float pv = Pf[16 * k];
            const float2 v = float2{acc[k].x / pv, acc[k].y / pv};
            if (mode & 2)
                __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, v),
                                            reinterpret_cast<unsigned long long *>(o + out_pos(b - 1, K)));
            else o[out_pos(b - 1, K)] = v;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int b = b0 + 16 * k;
            if (b > 0) o[b - 1] = acc[k];
        }
    }
}

template <bool NT, int SCHED, int WAVES, int DBG = 0, bool PERSIST = false, bool SYNC = false>
__device__ __forceinline__ void mrc_body(const float2 *__restrict__ iq, int S, int R, int prefix,
                                         const float2 *__restrict__ Hc, const float *__restrict__ P,
                                         float2 *__restrict__ out, long long nq, long long nblocks,
                                         long long per_xcd, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw = lds;
    const int w = threadIdx.x >> 6;
    const int t = threadIdx.x & 63;
    float2 *T = lds + TWBUF + w * TBUF;
    if (!PERSIST) {
        const long long pb = blockIdx.x;
        const long long lb = (pb & 7) * per_xcd + (pb >> 3);  // XCD-grouped logical block
        if (lb >= nblocks) return;
        fill_twiddles(tw);
        __syncthreads();
        const long long q = lb * WAVES + w;
        if (SYNC) {  // every wave takes part in the per-row barriers
            mrc_symbol<NT, SCHED, DBG, true>(iq, S, R, prefix, Hc, P, out, q < nq ? q : nq - 1,
                                             mode, t, T, tw, q < nq);
            return;
        }
        if (q >= nq) return;  // whole wave idle; no block-level sync follows
        mrc_symbol<NT, SCHED, DBG>(iq, S, R, prefix, Hc, P, out, q, mode, t, T, tw);
    } else {
        fill_twiddles(tw);
        __syncthreads();
        // XCD x (blocks b = x + 8 i) owns groups [x*per_xcd, (x+1)*per_xcd)
        const int x = blockIdx.x & 7;
        const long long i = blockIdx.x >> 3, nb_x = (gridDim.x + 7 - x) / 8;
        const long long g0 = x * per_xcd, g1 = min(nblocks, g0 + per_xcd);
        for (long long g = g0 + i; g < g1; g += nb_x) {
            const long long q = g * WAVES + w;
            if (q < nq) mrc_symbol<NT, SCHED, DBG>(iq, S, R, prefix, Hc, P, out, q, mode, t, T, tw);
        }
    }
}

// ---------------------------------------------------------------------------
// MRC with the channel estimates staged in LDS (HLDS): the 8 waves of a
// workgroup walk the antenna rows in lockstep; each thread prefetches 16 B of
// the next Hc row into a register before the FFT, the workgroup stores the
// row to LDS once and every wave reads its 16 values from there -- one
// dwordx4 per thread per row instead of eight per lane, and only LDS latency
// in front of the MAC.  LDS per workgroup is exactly 80 KiB (2 per CU):
//   TW1s [15][64] W1024^(c k2), k2 = 1..15     7680 B (k2-major: conflict free)
//   TW2s [16][4]  g(a) W64^(a k')                512 B
//   T    8 x [16][68] transpose images        69632 B (pitch 68: conflict free)
//   Hfree  Hc float4s 0..255                    4096 B
// and Hc float4s 256..511 live in the 16 unused 4-float2 row tails of the
// 8 transpose images (never touched by the transposes).  Both halves are
// read with per-lane affine addresses and no bank conflicts.
// ---------------------------------------------------------------------------


// HW = 16 (1024-thread workgroups, one per CU, 144 KiB of LDS): the 16
// transpose images' row tails hold the whole 8 KiB Hc row (512 float4), so
// float4 j lives at image j>>5, row (j>>1)&15, tail half j&1 -- and lane t's
// eight words j = t + 64 i are one affine stride of 2 images (TS float4s).
// Half the Hc L2 traffic and half the per-row barriers per symbol.
template <int HW>
constexpr size_t hlds_lds_bytes() {
    return (hlds::TW1S + hlds::TW2S + HW * hlds::TS) * sizeof(float2) + (HW == 8 ? 256 * sizeof(float4) : 0);
}
static_assert(hlds_lds_bytes<8>() == hlds::LDS_BYTES, "8-wave layout");
static_assert(hlds_lds_bytes<16>() <= 160 * 1024, "16-wave layout fits one CU");
template <int HW>
__device__ __forceinline__ float4 *hslot_hw(float2 *T0, float4 *hfree, int j) {
    if constexpr (HW == 16)
        return reinterpret_cast<float4 *>(T0 + (j >> 5) * hlds::TS + ((j >> 1) & 15) * hlds::TP + 64 +
                                          2 * (j & 1));
    else
        return hlds::hslot(T0, hfree, j);
}

// One antenna row of the PF loop: a[] holds this row on entry and the next
// row (`next`, when PREF) on exit.
template <bool NT, bool PREF, int PK, int HW = 8>
__device__ __forceinline__ void hlds_row_pf(const float2 *next, const float4 *hrow, int t, float2 (&a)[16],
                                            float2 *T, const float2 *tw1, const float2 *tw2,
                                            const float4 *lo, const float4 *hi, float4 *mine,
                                            float2 (&acc)[16]) {
    using namespace hlds;
    float2 x[16];
    row_fft_a<PK>(a, t, T, tw1);
    // a row is 512 float4 = 1024 float2: 1024 threads move 8 B each
    using HV = typename std::conditional<HW == 16, float2, float4>::type;
    const HV hreg = reinterpret_cast<const HV *>(hrow)[threadIdx.x];
    __builtin_amdgcn_sched_barrier(0);
    if (PREF) row_load<NT>(next, t, a);
    row_fft_b<PK>(t, T, tw2, x);
    lds_barrier();  // every wave is done with the previous Hc row
    *reinterpret_cast<HV *>(mine) = hreg;
    lds_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        // HW 8: 2 images = TS float4s; HW 16: hi = lo + 4 TS (ds_read offsets < 64 KiB)
        const float4 v = i < 4 ? lo[i * (HW == 16 ? TS : 64)] : hi[(i - 4) * TS];
        if constexpr (PK & 4) {
            pk::v2f a0 = pk::V(acc[2 * i]), a1 = pk::V(acc[2 * i + 1]);
            pk::mac(a0, pk::V(x[2 * i]), (pk::v2f){v.x, v.y});
            pk::mac(a1, pk::V(x[2 * i + 1]), (pk::v2f){v.z, v.w});
            acc[2 * i] = pk::F(a0);
            acc[2 * i + 1] = pk::F(a1);
            continue;
        }
        acc[2 * i].x = acc[2 * i].x + (x[2 * i].x * v.x - x[2 * i].y * v.y);
        acc[2 * i].y = acc[2 * i].y + (x[2 * i].x * v.y + x[2 * i].y * v.x);
        acc[2 * i + 1].x = acc[2 * i + 1].x + (x[2 * i + 1].x * v.z - x[2 * i + 1].y * v.w);
        acc[2 * i + 1].y = acc[2 * i + 1].y + (x[2 * i + 1].x * v.w + x[2 * i + 1].y * v.z);
    }
}

// Antenna-row loop of the HLDS kernel.  SHARED: the workgroup's 8 symbols
// share one frame and the Hc row goes through LDS; otherwise (a workgroup
// straddling a frame boundary) each wave loads its own Hc row from L2.
// PF (SHARED only): the next row's IQ is loaded into a[] as soon as the first
// FFT half has written a[] to the transpose image, so it is in flight during
// the second FFT half, the Hc exchange and the MAC (no extra registers: a[]
// is dead there).  The Hc prefetch is issued first: vmcnt retires in order.
template <bool NT, bool SHARED, bool PF, int PK = 0, int HW = 8>
__device__ __forceinline__ void hlds_rows(const float2 *sym, int Cp, int R, const float4 *Hf, int t,
                                          float2 *T, const float2 *tw1, const float2 *tw2,
                                          float2 *T0, float4 *hfree, float2 (&acc)[16]) {
    using namespace hlds;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = float2{0.f, 0.f};
    if constexpr (SHARED && PF) {
        float2 a[16];
        row_load<NT>(sym, t, a);
        const float4 *lo = HW == 16 ? hslot_hw<16>(T0, hfree, t) : hfree + t;
        const float4 *hi = HW == 16 ? lo + 4 * TS : hslot_hw<HW>(T0, hfree, 256 + t);
        // HW 16: thread i moves float2 i = half (i & 1) of float4 i >> 1
        float4 *mine = HW == 16 ? reinterpret_cast<float4 *>(reinterpret_cast<float2 *>(
                                      hslot_hw<16>(T0, hfree, threadIdx.x >> 1)) + (threadIdx.x & 1))
                                : hslot_hw<HW>(T0, hfree, threadIdx.x);
        // the last row is peeled so that the prefetch is unconditional: the
        // wait for the Hc word before the exchange is then vmcnt(16), not 0
        for (int r = 0; r + 1 < R; ++r)
            hlds_row_pf<NT, true, PK, HW>(sym + (long long)(r + 1) * Cp, Hf + (long long)r * (C / 2), t, a,
                                          T, tw1, tw2, lo, hi, mine, acc);
        hlds_row_pf<NT, false, PK, HW>(sym, Hf + (long long)(R - 1) * (C / 2), t, a, T, tw1, tw2, lo, hi,
                                       mine, acc);
        return;
    }
    static_assert(!SHARED || PF || HW == 8, "the 16-wave kernel stages Hc with PF only");
    for (int r = 0; r < R; ++r) {
        float2 a[16], x[16], h[16];
        row_load<NT>(sym + (long long)r * Cp, t, a);
        row_fft_a(a, t, T, tw1);
        if constexpr (SHARED) {
            // prefetch 16 B of the Hc row once a[] is dead: its latency
            // hides behind the second half of the FFT
            const float4 hreg = Hf[(long long)r * (C / 2) + threadIdx.x];
            row_fft_b(t, T, tw2, x);
            __syncthreads();  // every wave is done with the previous Hc row
            *hslot(T0, hfree, threadIdx.x) = hreg;
            __syncthreads();
            const float4 *lo = hfree + t;
            const float4 *hi = hslot(T0, hfree, 256 + t);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float4 v = i < 4 ? lo[i * 64] : hi[(i - 4) * TS];  // 2 images = TS float4s
                h[2 * i] = float2{v.x, v.y};
                h[2 * i + 1] = float2{v.z, v.w};
            }
        } else {
            row_fft_b(t, T, tw2, x);
            __builtin_amdgcn_sched_barrier(0);
            hc_load(Hf + (long long)r * (C / 2), t, h);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            acc[k].x = acc[k].x + (x[k].x * h[k].x - x[k].y * h[k].y);
            acc[k].y = acc[k].y + (x[k].x * h[k].y + x[k].y * h[k].x);
        }
    }
}

// HW waves (= HW consecutive data symbols) per workgroup.  align != 0:
// workgroups never straddle frames -- frame f owns logical blocks
// [f*bpf, (f+1)*bpf), bpf = ceil((S-1)/HW), so every workgroup stages its
// Hc rows through LDS (the last block of a frame has idle waves) -- instead
// of packing symbols densely and falling back to per-wave L2 loads of Hc in
// the workgroups that straddle two frames.
template <bool NT, bool PF, int PK, int HW = 8, bool ALIGN = false>
__global__ void __attribute__((amdgpu_flat_work_group_size(64 * HW, 64 * HW), amdgpu_waves_per_eu(4, 4)))
k_mrc_td1024_hlds(const float2 *__restrict__ iq, int S, int R, int prefix,
                  const float2 *__restrict__ Hc, const float *__restrict__ P,
                  float2 *__restrict__ out, long long nq, long long nblocks, long long per_xcd,
                  int mode) {
    using namespace hlds;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw1 = lds, *tw2 = lds + TW1S;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    float2 *T = lds + TW1S + TW2S + w * TS;
    float2 *T0 = lds + TW1S + TW2S;
    float4 *hfree = reinterpret_cast<float4 *>(T0 + HW * TS);
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);  // XCD-grouped logical block
    if (lb >= nblocks) return;
    // mode bit 3 (OFDM_MRC_PRIO=1, A/B): the second-dispatched half of the
    // workgroup at priority 1 (MI355X_MICROARCH.md, two waves per SIMD, item 4)
    if ((mode & 8) && w >= HW / 2) __builtin_amdgcn_s_setprio(1);
    fill(tw1, tw2);
    __syncthreads();

    // every wave takes part in the per-row barriers: tail waves duplicate the
    // last symbol and do not store
    const int nsym = S - 1;
    long long q, f, f0;
    bool store, shared;
    if constexpr (ALIGN) {
        const long long bpf = (nsym + HW - 1) / HW;
        f = lb / bpf;
        const int j = (int)(lb - f * bpf) * HW + w;  // symbol index within the frame
        store = j < nsym;
        q = f * nsym + (store ? j : nsym - 1);
        f0 = f;
        shared = true;
    } else {
        const long long qw = lb * HW + w;
        store = qw < nq;
        q = store ? qw : nq - 1;
        // the workgroup's Hc rows come from the frame of its first symbol; a
        // workgroup straddling two frames falls back to per-wave L2 loads
        f = q / nsym;
        f0 = (lb * HW) / nsym;
        const long long fl = ((lb * HW + HW - 1 < nq ? lb * HW + HW - 1 : nq - 1)) / nsym;
        shared = (f0 == fl);
    }
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const float4 *Hf = reinterpret_cast<const float4 *>(Hc + f * (long long)R * C);
    const float4 *Hf0 = reinterpret_cast<const float4 *>(Hc + f0 * (long long)R * C);

    float2 acc[16];
    if (shared)
        hlds_rows<NT, true, PF, PK, HW>(sym, Cp, R, Hf0, t, T, tw1, tw2, T0, hfree, acc);
    else
        hlds_rows<NT, false, false, 0, HW>(sym, Cp, R, Hf, t, T, tw1, tw2, T0, hfree, acc);
    if (!store) return;
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    if ((mode & 4) == 0) {
        // Stage the K outputs in this wave's transpose image (free after the
        // last row; its padding tails still hold other waves' Hc words, so
        // index it as [16][TP]) at their final positions, then store them as
        // 16 contiguous 512-B wave stores instead of 4 scattered 128-B runs
        // per instruction.
        const float *Pf = P + f * C + b0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int b = b0 + 16 * k;
            if (b == 0) continue;
            float2 v = acc[k];
            int j = b - 1;
            if ((mode & 1) == 0) {
                const float pv = Pf[16 * k];
                v = float2{acc[k].x / pv, acc[k].y / pv};
                j = out_pos(b - 1, K);
            }
            T[(j >> 6) * hlds::TP + (j & 63)] = v;
        }
        wave_lds_sync();
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const int j = t + 64 * m;
            if (j < K) o[j] = T[m * hlds::TP + t];
        }
        return;
    }
    if ((mode & 1) == 0) {
        const float *Pf = P + f * C + b0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int b = b0 + 16 * k;
            if (b == 0) continue;
            const float pv = Pf[16 * k];
            const float2 v = float2{acc[k].x / pv, acc[k].y / pv};
            if (mode & 2)
                __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, v),
                                            reinterpret_cast<unsigned long long *>(o + out_pos(b - 1, K)));
            else o[out_pos(b - 1, K)] = v;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int b = b0 + 16 * k;
            if (b > 0) o[b - 1] = acc[k];
        }
    }
}

// Small batches (k_mrc_td1024_rsplit): the 8 waves of a workgroup are 4
// symbols x 2 antenna halves -- wave w takes symbol w & 3 and rows
// [h R0, h R0 + R_h), h = w >> 2, R0 = ceil(R / 2), with its own Hc rows
// from L2 (the per-wave path of hlds_rows) -- and the two partial sums meet
// in LDS: Z = sum_{r < R0} + sum_{r >= R0} (not the strictly sequential
// antenna order of matrixMultThenSum; the difference is f32 rounding, far
// inside the 1e-5 tolerance).  Twice the waves per symbol, half the rows
// each: a batch of Q symbols is 2Q half-length wave tasks, so the last
// round of workgroups is much fuller when Q is only a few times the ~4 096
// resident waves (configs[1]: 10 000 symbols = 2.44 rounds of the 8-symbol
// workgroups, the third 44 % full).
template <bool NT>
__global__ void __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4)))
k_mrc_td1024_rsplit(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
                    const float *__restrict__ P, float2 *__restrict__ out, long long nq, long long nblocks,
                    long long per_xcd, int mode) {
    using namespace hlds;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw1 = lds, *tw2 = lds + TW1S;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    float2 *T0 = lds + TW1S + TW2S;
    float2 *T = T0 + w * TS;
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);  // XCD-grouped logical block
    if (lb >= nblocks) return;                            // whole workgroup
    fill(tw1, tw2);
    __syncthreads();
    const int h = w >> 2, R0 = (R + 1) >> 1, rows = h ? R - R0 : R0;
    const long long qw = lb * 4 + (w & 3);
    const bool store = qw < nq;
    const long long q = store ? qw : nq - 1;  // tail waves compute a valid symbol, never store
    const int nsym = S - 1;
    const long long f = q / nsym;
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + ((f * S + s) * (long long)R + (long long)h * R0) * Cp + prefix;
    const float4 *Hf = reinterpret_cast<const float4 *>(Hc + (f * (long long)R + (long long)h * R0) * C);
    float2 acc[16];
    hlds_rows<NT, false, false, 0, 8>(sym, Cp, rows, Hf, t, T, tw1, tw2, T0, nullptr, acc);
    // second half -> its transpose image -> first half (same lane, same bins)
    if (h) {
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k * hlds::TP + t] = acc[k];
    }
    __syncthreads();
    if (h || !store) return;
    const float2 *Tp = T0 + (w + 4) * TS;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const float2 v = Tp[k * hlds::TP + t];
        acc[k] = float2{acc[k].x + v.x, acc[k].y + v.y};
    }
    // outputs staged in this wave's image, then 16 contiguous 512-B stores
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    const float *Pf = P + f * C + b0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int b = b0 + 16 * k;
        if (b == 0) continue;
        float2 v = acc[k];
        int j = b - 1;
        if ((mode & 1) == 0) {
            const float pv = Pf[16 * k];
            v = float2{acc[k].x / pv, acc[k].y / pv};
            j = out_pos(b - 1, K);
        }
        T[(j >> 6) * hlds::TP + (j & 63)] = v;
    }
    wave_lds_sync();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int j = t + 64 * m;
        if (j < K) o[j] = T[m * hlds::TP + t];
    }
}

#define OFDM_MRC_ARGS                                                                            \
    const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,     \
        const float *__restrict__ P, float2 *__restrict__ out, long long nq, long long nblocks, \
        long long per_xcd, int mode
// 4 waves per workgroup: occupancy left to the compiler (LDS: 3 groups/CU)
template <bool NT, int SCHED>
__global__ void __launch_bounds__(256) k_mrc_td1024(OFDM_MRC_ARGS) {
    mrc_body<NT, SCHED, 4>(iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd, mode);
}
// 8 waves per workgroup, register budget for 4 waves/SIMD (2 groups/CU)
template <bool NT, int SCHED, int DBG = 0, bool PERSIST = false, bool SYNC = false>
__global__ void __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4)))
k_mrc_td1024_w8(OFDM_MRC_ARGS) {
    mrc_body<NT, SCHED, 8, DBG, PERSIST, SYNC>(iq, S, R, prefix, Hc, P, out, nq, nblocks, per_xcd,
                                               mode);
}
#undef OFDM_MRC_ARGS

}  // namespace td1024

hipError_t launch_ls_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial, hipStream_t s) {
    using namespace td1024;
    if (nframes <= 0) return hipSuccess;
    const size_t lds = (TWBUF + LS_WAVES * TBUF) * sizeof(float2);
    hipLaunchKernelGGL(k_ls_td1024, dim3((unsigned)nframes), dim3(64 * LS_WAVES), lds, s, iq, S, R, prefix, X, Hc,
                       P, partial);
    return hipGetLastError();
}

hipError_t launch_mrc_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode,
                             hipStream_t s) {
    using namespace td1024;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    // A/B switches, re-read on every launch so one process can compare them
    // (defaults = the measured best): OFDM_MRC_NT=0/1 plain / non-temporal IQ
    // loads, OFDM_MRC_SCHED=0/1 row-loop schedule, OFDM_MRC_WAVES=4/8 waves
    // per workgroup, OFDM_MRC_PERSIST=0/1 one workgroup per symbol group /
    // persistent grid (8-wave only), OFDM_MRC_SYNC=1 barrier per antenna row,
    // OFDM_MRC_HLDS=0/1 Hc rows staged in LDS per workgroup (8-wave), OFDM_MRC_DEBUG=1|2|3|4|7 diagnostic variants
    // (bit 0 no FFT, bit 1 no Hc, bit 2 no output stores)
    // (wrong results) pricing the memory side: 1 no FFT, 2 no Hc, 3 neither.
    auto knob = [](const char *n, int d) { const char *e = getenv(n); return e ? atoi(e) : d; };
    const int nt = knob("OFDM_MRC_NT", 1), sched = knob("OFDM_MRC_SCHED", 1);
    const int W = knob("OFDM_MRC_WAVES", 8) == 4 ? 4 : 8;
    const int persist = knob("OFDM_MRC_PERSIST", 0), dbg = knob("OFDM_MRC_DEBUG", 0);
    const int sync = knob("OFDM_MRC_SYNC", 0), hlds_on = knob("OFDM_MRC_HLDS", 1);
    if (knob("OFDM_MRC_NTSTORE", 0)) mode |= 2;  // bit 1: nontemporal output stores
    if (!knob("OFDM_MRC_OSTAGE", 1)) mode |= 4;  // bit 2: HLDS stores outputs without LDS staging
    if (knob("OFDM_MRC_PRIO", 0)) mode |= 8;     // bit 3: HLDS younger half at s_setprio 1
    const long long nblocks = (nq + W - 1) / W;
    const long long per_xcd = (nblocks + 7) / 8;
    long long grid = per_xcd * 8;
    if (W == 8 && persist) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess)
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const long long pg = (long long)cus * 2;  // 2 resident 8-wave groups per CU
        grid = pg < grid ? pg : grid;
    }
    if (grid > 0x7fffffffll) return hipErrorInvalidValue;
    // OFDM_MRC_RSPLIT=1: antenna-split workgroups (k_mrc_td1024_rsplit)
    if (W == 8 && hlds_on && !persist && !sync && !dbg && nt && knob("OFDM_MRC_RSPLIT", 0) == 1) {
        const long long nb = (nq + 3) / 4, pxcd = (nb + 7) / 8;
        if (pxcd * 8 > 0x7fffffffll) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_mrc_td1024_rsplit<true>), dim3((unsigned)(pxcd * 8)), dim3(512), hlds::LDS_BYTES, s,
                           iq, S, R, prefix, Hc, P, out, nq, nb, pxcd, mode);
        return hipGetLastError();
    }
    if (W == 8 && hlds_on && !persist && !sync && !dbg) {
        const int pf = knob("OFDM_MRC_PF", 1);  // next-row prefetch into the dead a[]
        // packed-f32 FFT halves / MAC (pk.hpp): bit 0 first FFT half, bit 1
        // second half, bit 2 MAC
        const int pkm = knob("OFDM_PK", 0);  // measured: no gain at C = 1024 (memory-bound), spills with PF
        // OFDM_MRC_ALIGN=1: frame-aligned workgroups; OFDM_MRC_HW=16: 16-wave
        // workgroups (one per CU, Hc row in the transpose-image tails)
        const int align = knob("OFDM_MRC_ALIGN", 0);
        const int hw = knob("OFDM_MRC_HW", 8) == 16 && nt && pf && pkm == 0 ? 16 : 8;
        const long long nsym = S - 1, bpf = (nsym + hw - 1) / hw;
        const long long nb = align && nt && pf && pkm == 0 ? nframes * bpf : (nq + hw - 1) / hw;
        const long long pxcd = (nb + 7) / 8;
        if (pxcd * 8 > 0x7fffffffll) return hipErrorInvalidValue;
        if (hw == 16) {
            for (const void *k : {reinterpret_cast<const void *>(&k_mrc_td1024_hlds<true, true, 0, 16, false>),
                                  reinterpret_cast<const void *>(&k_mrc_td1024_hlds<true, true, 0, 16, true>)}) {
                hipError_t e = opt_in_lds(k, (int)hlds_lds_bytes<16>());
                if (e != hipSuccess) return e;
            }
            if (align)
                hipLaunchKernelGGL((k_mrc_td1024_hlds<true, true, 0, 16, true>), dim3((unsigned)(pxcd * 8)),
                                   dim3(1024), hlds_lds_bytes<16>(), s, iq, S, R, prefix, Hc, P, out, nq, nb,
                                   pxcd, mode);
            else
                hipLaunchKernelGGL((k_mrc_td1024_hlds<true, true, 0, 16, false>), dim3((unsigned)(pxcd * 8)),
                                   dim3(1024), hlds_lds_bytes<16>(), s, iq, S, R, prefix, Hc, P, out, nq, nb,
                                   pxcd, mode);
            return hipGetLastError();
        }
#define OFDM_HLDS_LAUNCH(NTV, PFV, PKV)                                                             \
    hipLaunchKernelGGL((k_mrc_td1024_hlds<NTV, PFV, PKV>), dim3((unsigned)(pxcd * 8)), dim3(512),   \
                       hlds::LDS_BYTES, s, iq, S, R, prefix, Hc, P, out, nq, nb, pxcd, mode)
        if (align && nt && pf && pkm == 0) {
            hipLaunchKernelGGL((k_mrc_td1024_hlds<true, true, 0, 8, true>), dim3((unsigned)(pxcd * 8)), dim3(512),
                               hlds::LDS_BYTES, s, iq, S, R, prefix, Hc, P, out, nq, nb, pxcd, mode);
            return hipGetLastError();
        }
        if (nt && pf) {
            if (pkm == 7) OFDM_HLDS_LAUNCH(true, true, 7);
            else if (pkm == 3) OFDM_HLDS_LAUNCH(true, true, 3);
            else OFDM_HLDS_LAUNCH(true, true, 0);
        } else if (nt) {
            if (pkm == 7) OFDM_HLDS_LAUNCH(true, false, 7);
            else if (pkm == 3) OFDM_HLDS_LAUNCH(true, false, 3);
            else OFDM_HLDS_LAUNCH(true, false, 0);
        } else if (pf) OFDM_HLDS_LAUNCH(false, true, 0);
        else OFDM_HLDS_LAUNCH(false, false, 0);
#undef OFDM_HLDS_LAUNCH
        return hipGetLastError();
    }
    const size_t lds = (TWBUF + W * TBUF) * sizeof(float2);
#define OFDM_MRC_LAUNCH(KER, ...)                                                                  \
    hipLaunchKernelGGL((KER<__VA_ARGS__>), dim3((unsigned)grid), dim3(64 * W), lds, s, iq, S, R,   \
                       prefix, Hc, P, out, nq, nblocks, per_xcd, mode)
    if (W == 8 && persist) {
        if (dbg == 1) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 1, true);
        else if (dbg == 2) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 2, true);
        else if (dbg == 3) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 3, true);
        else if (nt) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 0, true);
        else OFDM_MRC_LAUNCH(k_mrc_td1024_w8, false, NOPREFETCH, 0, true);
    } else if (W == 8 && sync) {
        OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 0, false, true);
    } else if (W == 8) {
        if (dbg == 1) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 1);
        else if (dbg == 2) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 2);
        else if (dbg == 3) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 3);
        else if (dbg == 4) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 4);
        else if (dbg == 7) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH, 7);
        else if (nt) { if (sched) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, NOPREFETCH); else OFDM_MRC_LAUNCH(k_mrc_td1024_w8, true, PREFETCH_COPY); }
        else    { if (sched) OFDM_MRC_LAUNCH(k_mrc_td1024_w8, false, NOPREFETCH); else OFDM_MRC_LAUNCH(k_mrc_td1024_w8, false, PREFETCH_COPY); }
    } else {
        if (nt) { if (sched) OFDM_MRC_LAUNCH(k_mrc_td1024, true, NOPREFETCH); else OFDM_MRC_LAUNCH(k_mrc_td1024, true, PREFETCH_COPY); }
        else    { if (sched) OFDM_MRC_LAUNCH(k_mrc_td1024, false, NOPREFETCH); else OFDM_MRC_LAUNCH(k_mrc_td1024, false, PREFETCH_COPY); }
    }
#undef OFDM_MRC_LAUNCH
    return hipGetLastError();
}

}  // namespace ofdm
