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
//   k_mrc_td1024_hlds one wave (64 lanes) per data symbol, 8 per workgroup:
//                for every antenna row a 1024-point FFT in registers + one
//                LDS transpose, then acc += Y * Hc in registers (the Hc row
//                staged in LDS once per workgroup, the next IQ row
//                prefetched); finally acc / P stored at the rotated output
//                position.
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
#include "diag.hpp"

OFDM_DIAG_TU(td1024)


namespace ofdm {
namespace td1024 {

// ---------------------------------------------------------------------------
// LS: one workgroup (NW waves) per frame; wave w takes antenna rows w, w+NW,
// ... and keeps a partial |H|^2 per bin; partials are added in wave order
// through LDS (deterministic; for R <= NW this is findDistSqrd's sequential
// antenna order, cpuLS.hpp:211-228).  partial != 0: antenna-split mode (DC
// slot of P = 0).  P is written bin-indexed [F][C]; Hc lane-ordered
// [F][R][8][64] float4.  NW = 4 for large batches; NW = 16 (one antenna row
// per wave up to R = 16, 148 KiB of LDS) when the batch has too few frames to
// fill the GPU with 4-wave workgroups (BASELINE configs[1]: 100 frames x 16
// antennas -- the frame's rows are transformed side by side instead of four
// after one another).
// ---------------------------------------------------------------------------
constexpr int LS_WAVES = 4;

template <int NW>
__global__ void __launch_bounds__(64 * NW) k_ls_td1024(const float2 *__restrict__ iq, int S, int R,
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
    for (int r = w; r < R; r += NW) {
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
    float *pp = reinterpret_cast<float *>(lds + TWBUF);  // [NW][C], reuses T
    static_assert(NW * C * sizeof(float) <= NW * TBUF * sizeof(float2), "partials fit the transpose images");
#pragma unroll
    for (int k = 0; k < 16; ++k) pp[w * C + b0 + 16 * k] = p[k];
    __syncthreads();
    float *Pf = P + f * C;
    const int nw = R < NW ? R : NW;  // waves that hold rows
    for (int b = threadIdx.x; b < C; b += blockDim.x) {
        float sum = pp[b];
        for (int i = 1; i < nw; ++i) sum = sum + pp[i * C + b];
        Pf[b] = b == 0 ? (partial ? 0.f : 1.f) : sum;
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


// One antenna row of the prefetching loop: a[] holds this row on entry and
// the next row (`next`, when PREF) on exit.
template <bool PREF>
__device__ __forceinline__ void hlds_row_pf(const float2 *next, const float4 *hrow, int t, float2 (&a)[16],
                                            float2 *T, const float2 *tw1, const float2 *tw2,
                                            const float4 *lo, const float4 *hi, float4 *mine,
                                            float2 (&acc)[16]) {
    using namespace hlds;
    float2 x[16];
    row_fft_a(a, t, T, tw1);
    // a row is 512 float4: each of the 512 threads moves 16 B
    const float4 hreg = hrow[threadIdx.x];
    __builtin_amdgcn_sched_barrier(0);
    if (PREF) row_load<true>(next, t, a);
    row_fft_b(t, T, tw2, x);
    lds_barrier();  // every wave is done with the previous Hc row
    *mine = hreg;
    lds_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float4 v = i < 4 ? lo[i * 64] : hi[(i - 4) * TS];  // 2 images = TS float4s
        // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
        acc[2 * i].x = acc[2 * i].x + (x[2 * i].x * v.x - x[2 * i].y * v.y);
        acc[2 * i].y = acc[2 * i].y + (x[2 * i].x * v.y + x[2 * i].y * v.x);
        acc[2 * i + 1].x = acc[2 * i + 1].x + (x[2 * i + 1].x * v.z - x[2 * i + 1].y * v.w);
        acc[2 * i + 1].y = acc[2 * i + 1].y + (x[2 * i + 1].x * v.w + x[2 * i + 1].y * v.z);
    }
}

// Antenna-row loop.  SHARED: the workgroup's 8 symbols share one frame and
// the Hc row goes through LDS, the next row's IQ is loaded into a[] as soon
// as the first FFT half has written a[] to the transpose image (in flight
// during the second half, the Hc exchange and the MAC; no extra registers).
// Otherwise (a workgroup straddling a frame boundary) each wave loads its
// own Hc row from L2.
// R0: row 0 is already in this wave's transpose image, DMA'd there at the
// workgroup's start (row0_dma) and landed (vmcnt drained, barrier passed).
template <bool R0>
__device__ __forceinline__ void row0(const float2 *sym, int t, const float2 *T, float2 (&a)[16]) {
    if constexpr (R0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA (the compiler does not count asm loads)
#pragma unroll
        for (int m = 0; m < 16; ++m) a[m] = T[t + 64 * m];
    } else {
        row_load<true>(sym, t, a);
    }
}
// Row 0 of this wave's symbol (8 KiB) into its transpose image by LDS-DMA:
// no registers held, in flight through the table fill (and the estimate
// wait of the one-launch kernel).  The image's row tails carry other waves'
// Hc words only from row 0's exchange on, after every wave has read row 0.
__device__ __forceinline__ void row0_dma(const float2 *sym, int t, float2 *T) {
    const char *src = reinterpret_cast<const char *>(sym) + t * 16;
    const unsigned dst = lds_addr(T);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma16(src + j * 1024, dst + j * 1024);
}

template <bool SHARED, bool R0 = false>
__device__ __forceinline__ void hlds_rows(const float2 *sym, int Cp, int R, const float4 *Hf, int t,
                                          float2 *T, const float2 *tw1, const float2 *tw2,
                                          float2 *T0, float4 *hfree, float2 (&acc)[16]) {
    using namespace hlds;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = float2{0.f, 0.f};
    if constexpr (SHARED) {
        float2 a[16];
        row0<R0>(sym, t, T, a);
        const float4 *lo = hfree + t;
        const float4 *hi = hslot(T0, hfree, 256 + t);
        float4 *mine = hslot(T0, hfree, threadIdx.x);
        // the last row is peeled so that the prefetch is unconditional: the
        // wait for the Hc word before the exchange is then vmcnt(16), not 0
        for (int r = 0; r + 1 < R; ++r)
            hlds_row_pf<true>(sym + (long long)(r + 1) * Cp, Hf + (long long)r * (C / 2), lane_here(), a, T, tw1,
                                   tw2, lo, hi, mine, acc);
        hlds_row_pf<false>(sym, Hf + (long long)(R - 1) * (C / 2), lane_here(), a, T, tw1, tw2, lo, hi, mine,
                           acc);
    } else {
        for (int r = 0; r < R; ++r) {
            float2 a[16], x[16], h[16];
            if (r == 0)
                row0<R0>(sym, t, T, a);
            else
                row_load<true>(sym + (long long)r * Cp, t, a);
            row_fft_a(a, t, T, tw1);
            row_fft_b(t, T, tw2, x);
            __builtin_amdgcn_sched_barrier(0);
            hc_load(Hf + (long long)r * (C / 2), t, h);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                acc[k].x = acc[k].x + (x[k].x * h[k].x - x[k].y * h[k].y);
                acc[k].y = acc[k].y + (x[k].x * h[k].y + x[k].y * h[k].x);
            }
        }
    }
}

// Epilogue of one symbol (mode 0: normalise by P): stage the K outputs in
// this wave's transpose image (free after the last row; its padding tails
// still hold other waves' Hc words, so index it as [16][TP]) at their final
// positions, then store them as 16 contiguous 512-B nontemporal wave stores
// instead of 4 scattered 128-B runs per instruction.
__device__ __forceinline__ void hlds_epilogue(const float2 (&acc)[16], const float *P, long long f, long long q,
                                              int t, float2 *T, float2 *__restrict__ out, int mode) {
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    const float *Pf = P + f * C + b0;
    // all 16 |H|^2 loads issued before the first use (under the DC-bin
    // condition the compiler issued them one at a time, each behind a
    // vmcnt(0) wait; neutral at 4 waves/SIMD)
    float pv[16];
    if ((mode & 1) == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) pv[k] = Pf[16 * k];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int b = b0 + 16 * k;
        float2 v = acc[k];
        int j = b - 1;
        if ((mode & 1) == 0) {
            // acc * (1 / P): one reciprocal (v_rcp_f32, 1 ulp) and two
            // products instead of two IEEE divisions (10 instructions each);
            // within 2 ulp of the reference's division (cpuLS.hpp:364-368)
            const float rp = __builtin_amdgcn_rcpf(pv[k]);
            v = float2{acc[k].x * rp, acc[k].y * rp};
            j = out_pos(b > 0 ? b - 1 : 0, K);
        }
        if (b > 0) T[(j >> 6) * hlds::TP + (j & 63)] = v;
    }
    wave_lds_sync();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int j = t + 64 * m;
        if (j < K) {
            const float2 v = T[m * hlds::TP + t];
            // nontemporal (streaming) stores: 2-3 % faster than plain ones
            __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, v),
                                        reinterpret_cast<unsigned long long *>(o + j));
        }
    }
}

// 8 waves = 8 consecutive data symbols per workgroup, XCD-grouped block order
// (blocks b and b+8 share an XCD under round-robin dispatch, so a frame's
// workgroups share its Hc rows in one L2; speed only, never correctness).
// mode 0: out[q][out_pos(j)] = acc / P;  mode 1: out[q][j] = acc (numerator).
template <bool R0>
__global__ void __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4)))
k_mrc_td1024_hlds(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
                  const float *__restrict__ P, float2 *__restrict__ out, long long nq, long long nblocks,
                  long long per_xcd, int mode) {
    using namespace hlds;
    constexpr int HW = WAVES;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw1 = lds, *tw2 = lds + TW1S;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    float2 *T = lds + TW1S + TW2S + w * TS;
    float2 *T0 = lds + TW1S + TW2S;
    float4 *hfree = reinterpret_cast<float4 *>(T0 + HW * TS);
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);  // XCD-grouped logical block
    if (lb >= nblocks) return;

    // every wave takes part in the per-row barriers: tail waves duplicate the
    // last symbol and do not store
    const int nsym = S - 1;
    const long long qw = lb * HW + w;
    const bool store = qw < nq;
    const long long q = store ? qw : nq - 1;
    // the workgroup's Hc rows come from the frame of its first symbol; a
    // workgroup straddling two frames falls back to per-wave L2 loads
    const long long f = q / nsym;
    const long long f0 = (lb * HW) / nsym;
    const long long fl = ((lb * HW + HW - 1 < nq ? lb * HW + HW - 1 : nq - 1)) / nsym;
    const int s = 1 + (int)(q % nsym);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    if constexpr (R0) row0_dma(sym, t, T);
    fill(tw1, tw2);
    __syncthreads();

    float2 acc[16];
    if (f0 == fl)
        hlds_rows<true, R0>(sym, Cp, R, reinterpret_cast<const float4 *>(Hc + f0 * (long long)R * C), t, T,
                                 tw1, tw2, T0, hfree, acc);
    else
        hlds_rows<false, R0>(sym, Cp, R, reinterpret_cast<const float4 *>(Hc + f * (long long)R * C), t, T,
                                tw1, tw2, T0, hfree, acc);
    if (!store) return;
    hlds_epilogue(acc, P, f, q, t, T, out, mode);
}


// ---------------------------------------------------------------------------
// One-launch frame demodulation (ofdm_frame_demod at C = 1024): the reference
// runs demodOneFrameCUDA as dependent launches (gpuLS.cu:575-675); here the
// LS of every frame and the MRC of every data symbol share ONE grid.
// Workgroups 0 .. nls-1 (nls = nframes rounded up to 8, so the MRC blocks
// keep their XCD grouping) each estimate one frame -- FFT of its R pilot
// rows, Hc = conj(Y/X) into the workspace in lane order, P = sum_r |Hc|^2 --
// and publish it with an agent-scope release and a 64-bit flag (cdna_hip_
// programming.md Guideline 16, R1: plain stores, every storing wave's
// vmcnt(0), barrier, one lane's release fence + vmcnt(0) + relaxed agent
// flag store).  The MRC workgroups behind them poll the flags of the (one or
// two) frames they read with one lane, relaxed, then ONE agent acquire, a
// vmcnt(0) and a barrier before any Hc / P load.  Flags hold a per-launch
// 64-bit epoch (never reused; a workspace's flags need no reset).  The wait
// is bounded: a workgroup that has not seen its flag after SPIN_TICKS of
// the 100 MHz wall clock estimates the frame itself (the same bytes) and
// goes on, so no dispatch-order or residency assumption is needed for a
// correct result -- in-order dispatch only makes the wait short.
// ---------------------------------------------------------------------------
// LS of frame f by one 8-wave workgroup in the HLDS LDS layout (tables
// filled): wave w takes rows w, w + 8, ...; partial |H|^2 added in wave
// order through the transpose images (the k_ls_td1024<8> order).
__device__ __forceinline__ void hlds_ls_frame(const float2 *__restrict__ iq, int S, int R, int prefix,
                                              const float2 *__restrict__ X, float2 *Hc, float *P, long long f,
                                              int w, int t, float2 *T, float2 *T0, const float2 *tw1,
                                              const float2 *tw2, unsigned long long *mx = nullptr) {
    using namespace hlds;
    (void)mx;  // diagnostic build: phase stamps
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
    for (int r = w; r < R; r += WAVES) {
        float2 a[16], x[16];
        const int tl = lane_here();
        row_load<true>(pilot + (long long)r * Cp, tl, a);
        row_fft_a(a, tl, T, tw1);
        row_fft_b(tl, T, tw2, x);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            float2 h = ls_conj(x[k], xp[k]);  // divideOneRow + conj (cpuLS.hpp:233-244)
            if (b0 + 16 * k == 0) h = float2{0.f, 0.f};
            x[k] = h;
            p[k] = p[k] + (h.x * h.x) + (h.y * h.y);
        }
        // hc_store's layout, write-through (sc1): visible at agent scope once vmcnt drains
#pragma unroll
        for (int i = 0; i < 8; ++i) store16_wt(Hf, R * C * 8, (r * (C / 2) + i * 64 + tl) * 16, x[2 * i], x[2 * i + 1]);
        if (r == w) {
            OFDM_DIAG_MARKP(mx, 1)
        }
    }
    OFDM_DIAG_MARKP(mx, 2)
    __syncthreads();  // every wave is done with its transpose image
    float *pp = reinterpret_cast<float *>(T0);  // [WAVES][C], over the images
#pragma unroll
    for (int k = 0; k < 16; ++k) pp[w * C + b0 + 16 * k] = p[k];
    __syncthreads();
    float *Pf = P + f * C;
    const int nw = R < WAVES ? R : WAVES;
    for (int b = threadIdx.x; b < C; b += blockDim.x) {
        float sum = pp[b];
        for (int i = 1; i < nw; ++i) sum = sum + pp[i * C + b];
        const float v = b == 0 ? 1.f : sum;
        store4_wt(Pf + b, v);
    }
    OFDM_DIAG_MARKP(mx, 3)
    __syncthreads();  // pp (the transpose images) read before they are reused
}

// A half unit of the one-launch demod's schedule tail: four consecutive data
// symbols q0 .. q0+3 with each symbol's antenna rows split over two waves
// (wave w: symbol w & 3, rows [0, R0) for w < 4, [R0, R) for w >= 4), so the
// unit takes about half a block's time.  Each wave reads its own Hc rows
// (L2; no shared row, the two halves of the workgroup are at different rows),
// the second-half waves hand their sums over through their transpose images
// and the first-half waves add them (first half + second half) and store.
// Every wave reaches the one workgroup barrier.
__device__ __forceinline__ void split_unit(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *Hc,
                                           const float *P, float2 *__restrict__ out, long long nq, long long q0, int w,
                                           int t, float2 *T, float2 *T0, const float2 *tw1, const float2 *tw2) {
    const int nsym = S - 1, Cp = C + prefix, hh = w >> 2, R0 = (R + 1) >> 1;
    const long long qw = q0 + (w & 3);
    const bool store = qw < nq;
    const long long q = store ? qw : nq - 1;
    const long long f = q / nsym;
    const int s = 1 + (int)(q % nsym);
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const float4 *Hf = reinterpret_cast<const float4 *>(Hc + f * (long long)R * C);
    float2 acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = float2{0.f, 0.f};
    const int r1 = hh ? R : R0;
    for (int r = hh ? R0 : 0; r < r1; ++r) {
        float2 a[16], x[16], h[16];
        row_load<true>(sym + (long long)r * Cp, t, a);
        hlds::row_fft_a(a, t, T, tw1);
        hlds::row_fft_b(t, T, tw2, x);
        __builtin_amdgcn_sched_barrier(0);
        hc_load(Hf + (long long)r * (C / 2), t, h);
#pragma unroll
        for (int k = 0; k < 16; ++k) {  // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order per half
            acc[k].x = acc[k].x + (x[k].x * h[k].x - x[k].y * h[k].y);
            acc[k].y = acc[k].y + (x[k].x * h[k].y + x[k].y * h[k].x);
        }
    }
    if (hh) {
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k * hlds::TP + t] = acc[k];
    }
    __syncthreads();
    if (hh) return;
    const float2 *Tp = T0 + (w + 4) * hlds::TS;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const float2 v = Tp[k * hlds::TP + t];
        acc[k] = float2{acc[k].x + v.x, acc[k].y + v.y};
    }
    if (store) hlds_epilogue(acc, P, f, q, t, T, out, 0);
}

// The estimate is stored write-through (sc1: 16-B Hc stores, 4-B agent
// atomic P stores) and published without a release fence, whose L2
// write-back would also flush the output lines the MRC workgroups of the
// same XCD left dirty (wave_fft1024.hpp: publish_flag / consume_flags;
// same-process A/B vs plain stores + release fence: equal to 1 % faster,
// DESIGN.md 4.6).
__global__ void __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4)))
k_demod_td1024(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ X, float2 *Hc,
               float *P, float2 *__restrict__ out, long long nq, long long nblocks, Tickets tk, long long k0, long long split, unsigned long long *flags, unsigned long long epoch,
               int nls, long long nframes, long long spin_ticks) {
    using namespace hlds;
    constexpr int HW = WAVES;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *tw1 = lds, *tw2 = lds + TW1S;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    float2 *T = lds + TW1S + TW2S + w * TS;
    float2 *T0 = lds + TW1S + TW2S;
    float4 *hfree = reinterpret_cast<float4 *>(T0 + HW * TS);
    OFDM_DIAG_BEGIN()

    // Frames this workgroup estimates itself, [e0, e1]: an estimator
    // workgroup its own frame; an MRC workgroup none, or -- when a flag it
    // waits for is not published within spin_ticks -- the frames it reads.
    // ONE call site of hlds_ls_frame for both, so that both run the same
    // inlined code and write the same bytes (two inlined copies
    // could contract differently).
    const bool estimator = (int)blockIdx.x < nls;
    // MRC workgroups: the logical block (8 consecutive data symbols) is a
    // work ticket (take_block: own XCD's range first, then the others'),
    // kept in SGPRs
    auto first_frame = [&](long long lb) { return (lb * HW) / (S - 1); };
    auto last_frame = [&](long long lb) { return ((lb * HW + HW - 1 < nq ? lb * HW + HW - 1 : nq - 1)) / (S - 1); };
    const int nsym = S - 1, Cp = C + prefix;
    // this wave's symbol of logical block lb (the last one for tail waves)
    auto sym_of = [&](long long lb) {
        const long long qw = lb * HW + w, q = qw < nq ? qw : nq - 1;
        return iq + ((q / nsym) * S + 1 + q % nsym) * (long long)R * Cp + prefix;
    };
    long long e0 = 1, e1 = 0, lb = 0;
    int um = 0;  // unit mode: 0 the whole block, 1 / 2 its first / second four symbols, rows split over waves
    if (estimator) {
        e0 = e1 = blockIdx.x;
        if (e0 >= nframes) return;
        // the estimates are the first round's critical path: the estimator
        // waves issue ahead of receiver waves on the same SIMDs (same process,
        // configs[1] 0.295 -> 0.292 ms on one box, equal on another;
        // profiles/r6/r6s_*, r6t_*)
        __builtin_amdgcn_s_setprio(3);
        fill(tw1, tw2);
        __syncthreads();
        OFDM_DIAG_MARKN(0)
    } else {
        // the table loads first: in flight through the work ticket
        FillRegs fr;
        fill_load(fr);
        lb = wg_take_unit(tk, nblocks, k0, (long long)blockIdx.x - nls, split,
                          reinterpret_cast<long long *>(hfree + 255));
        if (lb < 0) return;  // every block taken
        OFDM_DIAG_MARKN(0)
        um = (int)(lb & 3);
        lb >>= 2;
        fill_store(tw1, tw2, fr);
        // then row 0 of the wave's symbol into its transpose image by LDS-DMA
        // and a first look at the estimate flags, in flight together: a
        // block's start costs about two memory round trips (ticket, then
        // DMA / flags), not four
        const long long f0 = first_frame(lb), fl = last_frame(lb);
        if (!um) row0_dma(sym_of(lb), t, T);
        bool seen_before = false;
        if (threadIdx.x == 0)
            seen_before = __hip_atomic_load((gu64 *)(flags + f0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch &&
                          __hip_atomic_load((gu64 *)(flags + fl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
        OFDM_DIAG_MARKN(1)
        // wait for the estimates of frames f0 .. fl (hfree, not used before
        // the rows, carries the outcome); not published in time: estimate
        // here (identical bytes) and read them back behind an acquire of our own
        if (!consume_flags(flags, f0, fl, epoch, spin_ticks, reinterpret_cast<int *>(hfree), seen_before)) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // row 0's DMA landed before the images are reused
            __syncthreads();
            e0 = f0;
            e1 = fl;
        }
    }
    for (long long ff = e0; ff <= e1; ++ff)
        hlds_ls_frame(iq, S, R, prefix, X, Hc, P, ff, w, t, T, T0, tw1, tw2, OFDM_DIAG_ARG);
    if (estimator) {
        OFDM_DIAG_MARK()
        publish_flag(flags + e0, epoch);
        OFDM_DIAG_END_SLOT(td1024, epoch);
        return;
    }
    if (e0 <= e1) {
        acquire_all();
        if (!um) row0_dma(sym_of(lb), t, T);  // the estimate used the images: row 0 again
    }
    OFDM_DIAG_MARK()

    if (um) {  // a half unit of the schedule's tail (launch_demod_td1024)
        split_unit(iq, S, R, prefix, Hc, P, out, nq, lb * HW + 4 * (um - 1), w, t, T, T0, tw1, tw2);
        OFDM_DIAG_END_SLOT(td1024, epoch);
        return;
    }
    const long long qw = lb * HW + w;
    const bool store = qw < nq;
    const long long q = store ? qw : nq - 1;
    const long long f = q / nsym;
    const long long f0 = first_frame(lb), fl = last_frame(lb);
    const float2 *sym = sym_of(lb);
    float2 acc[16];
    if (f0 == fl)
        hlds_rows<true, true>(sym, Cp, R, reinterpret_cast<const float4 *>(Hc + f0 * (long long)R * C), t, T,
                              tw1, tw2, T0, hfree, acc);
    else
        hlds_rows<false, true>(sym, Cp, R, reinterpret_cast<const float4 *>(Hc + f * (long long)R * C), t, T,
                               tw1, tw2, T0, hfree, acc);
    OFDM_DIAG_MARKN(2)
    if (store) hlds_epilogue(acc, P, f, q, lane_here(), T, out, 0);
    OFDM_DIAG_END_SLOT(td1024, epoch);
}

}  // namespace td1024

hipError_t launch_ls_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial, hipStream_t s) {
    using namespace td1024;
    if (nframes <= 0) return hipSuccess;
    if (nframes > 0x7fffffffll) return hipErrorInvalidValue;
    // 4-wave workgroups unless they leave the GPU under-filled: fewer than
    // 2 waves per SIMD (2048 waves) with rows left to spread
    int nw = (nframes * LS_WAVES < 2048 && R > LS_WAVES) ? 16 : LS_WAVES;
    auto k16 = k_ls_td1024<16>;
    auto k4 = k_ls_td1024<LS_WAVES>;
    auto k8 = k16;  // 8-wave workgroups: A/B build only
    if (nw == 16 || nw == 8) {
        auto kern = nw == 16 ? k16 : k8;
        const size_t lds = (TWBUF + nw * TBUF) * sizeof(float2);
        if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)lds); e != hipSuccess) return e;
        hipLaunchKernelGGL(kern, dim3((unsigned)nframes), dim3(64 * nw), lds, s, iq, S, R, prefix, X, Hc, P,
                           partial);
        return hipGetLastError();
    }
    const size_t lds = (TWBUF + LS_WAVES * TBUF) * sizeof(float2);
    hipLaunchKernelGGL(k4, dim3((unsigned)nframes), dim3(64 * LS_WAVES), lds, s, iq, S, R, prefix, X, Hc, P,
                       partial);
    return hipGetLastError();
}

hipError_t launch_mrc_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode,
                             hipStream_t s) {
    using namespace td1024;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    const long long nb = (nq + hlds::WAVES - 1) / hlds::WAVES;
    const long long pxcd = (nb + 7) / 8;
    if (pxcd * 8 > 0x7fffffffll) return hipErrorInvalidValue;
    // R0: each wave's row 0 DMA'd into its transpose image ahead of the table
    // fill (same process, bit-identical: R=16 x 100 frames 0.301 -> 0.293 ms,
    // R=64 x 400 3.961 -> 3.922; profiles/r3/r3p_row0_dma_ab.jsonl).  The
    // one-launch kernel takes it too since round 6, once its receivers ran
    // without scratch (profiles/r6/r6m2_*).
    auto kern = k_mrc_td1024_hlds<true>;
    hipLaunchKernelGGL(kern, dim3((unsigned)(pxcd * 8)), dim3(64 * hlds::WAVES), hlds::LDS_BYTES, s, iq, S, R,
                       prefix, Hc, P, out, nq, nb, pxcd, mode);
    return hipGetLastError();
}

// One-launch LS + MRC (ofdm_frame_demod, mode 0).  flags: nframes 64-bit
// words of the workspace; epoch: a value none of them holds (per launch);
// spin_ticks: how long (100 MHz ticks) an MRC workgroup waits for a frame's
// flag before it estimates the frame itself (< 0: SPIN_TICKS).
hipError_t launch_demod_td1024(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *X,
                               float2 *Hc, float *P, float2 *out, Tickets tk,
                               unsigned long long *flags, unsigned long long epoch, long long spin_ticks,
                               hipStream_t s) {
    using namespace td1024;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    const long long nb = (nq + hlds::WAVES - 1) / hlds::WAVES;
    const long long nls = (nframes + 7) / 8 * 8;
    // the first TWO rounds static (k0 = twice the XCD's resident workgroups
    // per XCD range: a second-round unit costs no ticket round trip before
    // its row 0 and flags are in flight; configs[1] 0.292 -> 0.280 ms, R = 64
    // x 100 frames 1.043 -> 1.008 ms, larger batches equal; 1.5 / 3 static
    // rounds 0.288 / 0.286 ms: profiles/r6/r6ag_*, r6ah_*), then work tickets
    // with the schedule's tail in half units: the last k1 blocks of every
    // XCD range (k1 = the XCD's resident workgroups) -- the last rounds end on
    // units of about half a block's time (R >= 2)
    const long long k1 = ticket_k0(2), k0 = 2 * k1, split = R >= 2 ? k1 : 0;
    const long long g = ticket_grid(nb, 8 * split);
    if (g + nls > 0x7fffffffll) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_demod_td1024, dim3((unsigned)(nls + g)), dim3(64 * hlds::WAVES), hlds::LDS_BYTES, s, iq,
                       S, R, prefix, X, Hc, P, out, nq, nb, tk, k0, split, flags, epoch, (int)nls, nframes,
                       spin_ticks < 0 ? SPIN_TICKS : spin_ticks);
    return hipGetLastError();
}

}  // namespace ofdm
