// frame_td4096.hip -- fused time-domain receiver for C = 4096 subcarriers
// (BASELINE configs[4]: 4096 subcarriers, 256 antennas split 32 per GPU).
//
// A 4096-point row is shared by a PAIR of waves.  Wave e (0 or 1) of the
// pair computes the bins X[2 k + e] by one decimation-in-frequency step:
//   y_e[n] = (x[n] + (-1)^e x[n + 2048]) W4096^(e n),  n < 2048
//   X[2 k + e] = FFT2048(y_e)[k]
// and FFT2048 is done as in frame_td2048.hip (u/v split in registers + two
// 1024-point wave FFTs).  Each wave reads the whole row; a workgroup barrier
// per antenna row keeps the two waves of a pair together so that the
// partner's read of the same 32 KiB hits L2 (without it the fabric carries
// every row twice: profiles/, PMC ratio 2.02) -- no LDS exchange needed.
// Lane (q, a) of wave e owns bins 4 b + e and 4 b + 2 + e, b = b0(t) + 16 k.
//
// Hc "lane order" for C = 4096: per (frame, antenna) 4096 float2 in planes
// [e][h][k >> 1][t][k & 1]: float2 e*2048 + h*1024 + (k >> 1)*128 + 2 t +
// (k & 1) = Hc[4 b + 2 h + e] with b = b0(t) + 16 k -- lane t's bins k and
// k + 1 side by side, so that the MRC kernel reads a plane from LDS as 8
// ds_read_b128 (4 LDS cycles each) instead of 8 ds_read2st64_b64 (8 each).
// P bin-indexed [F][C].  The LS kernel (one read per frame) uses the direct
// form above, each wave reading the whole row.
//
// The MRC kernel (k_mrc_td4096h) reads every row ONCE per pair: radix-4
// decimation in frequency, n = n0 + 1024 n1, z_c[n0] = sum_n1 x[n0 + 1024 n1]
// (-i)^(c n1) W4096^(c n0), X[4 k + c] = FFT1024(z_c)[k].  Wave e loads
// quarters e and e + 2 and forms s = x_e + x_(e+2), d = x_e - x_(e+2); the
// pair swaps one half through LDS (wave 0 sends d, wave 1 sends s), so wave 0
// holds a = x0 + x2, c = x1 + x3 -> z0 = a + c, z2 = (a - c) W^(2 n0), and
// wave 1 holds b = x0 - x2, d = x1 - x3 -> z1 = (b - i d) W^(n0),
// z3 = (b + i d) W^(3 n0).  Same bin ownership as above.
#include "launch.hpp"
#include "wave_fft1024.hpp"
#include "diag.hpp"

OFDM_DIAG_TU(td4096)

namespace ofdm {
namespace td4096 {

using td1024::lane_bin0;
using td1024::row_load;
namespace hl = td1024::hlds;

constexpr int C = 4096;
constexpr int K = C - 1;
constexpr int TWV = 16 * 64;  // W2048^(t + 64 m), m < 16, [m][t]
constexpr int TWE = 32 * 64;  // W4096^(t + 64 m), m < 32, [m][t]
// LDS: TW1s | TW2s | TWV | TWE | per-wave transpose images
constexpr int TAB = hl::TW1S + hl::TW2S + TWV + TWE;
constexpr size_t lds_bytes(int waves) { return (size_t)(TAB + waves * hl::TS) * sizeof(float2); }

__device__ __forceinline__ void fill_tables(float2 *lds) {
    hl::fill(lds, lds + hl::TW1S);
    float2 *twv = lds + hl::TW1S + hl::TW2S;
    for (int i = threadIdx.x; i < TWV; i += blockDim.x) {
        const int m = i / 64, t = i % 64;
        twv[i] = g_tw[(t + 64 * m) * (OFDM_TW_N / 2048)];
    }
    float2 *twe = twv + TWV;
    for (int i = threadIdx.x; i < TWE; i += blockDim.x) {
        const int m = i / 64, t = i % 64;
        twe[i] = g_tw[(t + 64 * m) * (OFDM_TW_N / C)];
    }
}

// wave e's half of the FFT of one 4096-sample row:
//   xe[k] = X[4 b + e], xo[k] = X[4 b + 2 + e]
template <int E, bool NT>
__device__ __forceinline__ void row_fft4096(const float2 *__restrict__ src, int t, float2 *T,
                                            const float2 *lds, float2 (&xe)[16], float2 (&xo)[16]) {
    const float2 *tw1 = lds, *tw2 = lds + hl::TW1S;
    const float2 *twv = lds + hl::TW1S + hl::TW2S, *twe = twv + TWV;
    float2 lo[16], hi[16];
    {
        float2 b[16];
        row_load<NT>(src, t, lo);
        row_load<NT>(src + 2048, t, b);
#pragma unroll
        for (int m = 0; m < 16; ++m)
            lo[m] = E ? cmul(csub(lo[m], b[m]), twe[m * 64 + t]) : cadd(lo[m], b[m]);
        row_load<NT>(src + 1024, t, hi);
        row_load<NT>(src + 3072, t, b);
#pragma unroll
        for (int m = 0; m < 16; ++m)
            hi[m] = E ? cmul(csub(hi[m], b[m]), twe[(m + 16) * 64 + t]) : cadd(hi[m], b[m]);
    }
    // FFT2048 of y = (lo, hi): u = lo + hi -> even bins, v = (lo - hi) W2048^n -> odd
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const float2 d = csub(lo[m], hi[m]);
        lo[m] = cadd(lo[m], hi[m]);
        hi[m] = cmul(d, twv[m * 64 + t]);
    }
    hl::row_fft_a(lo, t, T, tw1);
    hl::row_fft_b(t, T, tw2, xe);
    hl::row_fft_a(hi, t, T, tw1);
    hl::row_fft_b(t, T, tw2, xo);
}

// ---------------------------------------------------------------------------
// LS: one workgroup (4 wave pairs) per frame; pair j takes antenna rows j,
// j+4, ...  Pilots in LDS; partial |H|^2 per pair combined in pair order.
// 132 KiB of LDS, one workgroup per CU; round 1's 2-pair workgroups (98 KiB,
// also one per CU, so one wave per SIMD) took 29-41 % longer (0.318 vs
// 0.247 ms for 400 frames x 32 antennas; 0.134 vs 0.095 ms for 50).
// ---------------------------------------------------------------------------
constexpr int LS_WAVES = 8;
constexpr size_t ls_lds(int nw) { return lds_bytes(nw) + (size_t)C * sizeof(float2); }

template <int E, int LS_PAIRS>
__device__ __forceinline__ void ls_rows(const float2 *pilot, int Cp, int R, int j, int t, float2 *T,
                                        const float2 *lds, const float2 *xs, float2 *Hf, float *pp) {
    const int b0 = lane_bin0(t);
    float pe[16], po[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) pe[k] = po[k] = 0.f;
    for (int r = j; r < R; r += LS_PAIRS) {
        float2 xe[16], xo[16];
        row_fft4096<E, false>(pilot + (long long)r * Cp, t, T, lds, xe, xo);
        float4 *hr = reinterpret_cast<float4 *>(Hf + (long long)r * C + E * 2048);
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
            float2 he[2], ho[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int be = 4 * (b0 + 16 * (k + i)) + E;
                // divideOneRow + conj (cpuLS.hpp:233-244, 303-307); DC bin dropped
                he[i] = ls_conj(xe[k + i], xs[be]);
                if (be == 0) he[i] = float2{0.f, 0.f};
                ho[i] = ls_conj(xo[k + i], xs[be + 2]);
                pe[k + i] = pe[k + i] + (he[i].x * he[i].x) + (he[i].y * he[i].y);  // findDistSqrd order
                po[k + i] = po[k + i] + (ho[i].x * ho[i].x) + (ho[i].y * ho[i].y);
            }
            hr[(k >> 1) * 64 + t] = float4{he[0].x, he[0].y, he[1].x, he[1].y};
            hr[512 + (k >> 1) * 64 + t] = float4{ho[0].x, ho[0].y, ho[1].x, ho[1].y};
        }
    }
    __syncthreads();  // every wave is done with its transpose image (pp reuses it)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int be = 4 * (b0 + 16 * k) + E;
        pp[j * C + be] = pe[k];
        pp[j * C + be + 2] = po[k];
    }
}

// LS of frame f by an NW-wave workgroup (LS LDS layout, ls_lds(NW) bytes).
template <int NW = LS_WAVES>
__device__ __forceinline__ void ls_frame4096(const float2 *__restrict__ iq, int S, int R, int prefix,
                                             const float2 *__restrict__ X, float2 *Hc, float *P, long long f,
                                             float2 *lds, int partial) {
    constexpr int LS_PAIRS = NW / 2;
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float2 *T = lds + TAB + w * hl::TS;
    float2 *xs = lds + TAB + NW * hl::TS;  // xs[b] = X[b - 1], xs[0] unused
    fill_tables(lds);
    for (int b = threadIdx.x; b < C; b += blockDim.x) xs[b] = b ? X[b - 1] : float2{1.f, 0.f};
    __syncthreads();

    const int Cp = C + prefix;
    const float2 *pilot = iq + f * (long long)S * R * Cp + prefix;
    float2 *Hf = Hc + f * (long long)R * C;
    float *pp = reinterpret_cast<float *>(lds + TAB);  // [LS_PAIRS][C], reuses T
    if (w & 1)
        ls_rows<1, LS_PAIRS>(pilot, Cp, R, w >> 1, t, T, lds, xs, Hf, pp);
    else
        ls_rows<0, LS_PAIRS>(pilot, Cp, R, w >> 1, t, T, lds, xs, Hf, pp);
    __syncthreads();
    float *Pf = P + f * C;
    for (int b = threadIdx.x; b < C; b += blockDim.x) {
        float sum = pp[b];
        for (int i = 1; i < LS_PAIRS; ++i) sum = sum + pp[i * C + b];  // antennas in order
        const float v = b == 0 ? (partial ? 0.f : 1.f) : sum;
        Pf[b] = v;
    }
    __syncthreads();  // pp (the transpose images) read before they are reused
}

template <int NW = LS_WAVES>
__global__ void __launch_bounds__(64 * NW) k_ls_td4096(const float2 *__restrict__ iq, int S, int R,
                                                       int prefix, const float2 *__restrict__ X,
                                                       float2 *__restrict__ Hc, float *__restrict__ P,
                                                       int partial) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    ls_frame4096<NW>(iq, S, R, prefix, X, Hc, P, blockIdx.x, lds, partial);
}

// ---------------------------------------------------------------------------
// MRC, one read per row: a wave PAIR per data symbol (see the header: radix-4
// DIF, wave e loads quarters e and e + 2, the pair swaps one half through
// LDS).  The DIF twiddles W4096^(c n0), n0 = t + 64 m, are the lane's
// W4096^(c t) times the compile-time W64^(c m).  Packed-f32 arithmetic
// (pk.hpp) in the split, both FFT halves and the MAC.
// ---------------------------------------------------------------------------
constexpr int X_TAB = hl::TW1S + hl::TW2S;
// The MRC kernel's transpose images: hlds::TP16 pitch (16-B reads of the
// second FFT half, wave_fft1024.hpp)
constexpr int TP4 = hl::TP16;
constexpr int TS4 = hl::TS16;
using hl::fa_write16;
using hl::fb_read16;
using hl::perm16;

template <int CM, int M>
__device__ __forceinline__ pk::v2f dif_tw(pk::v2f base) {  // base * W64^(CM * M)
    if constexpr ((CM * M) % 64 == 0) return base;
    constexpr float2 w = tw_const<64, CM * M>();
    return pk::cmul_s_v(base, (pk::v2f){w.x, w.y});
}

using td1024::dma16;
using td1024::lds_addr;
using td1024::wg_take_block;

// One 32 KiB Hc row (4096 float2) into LDS by an NW-wave workgroup: 32 / NW
// wave-instructions of 1 KiB per wave, natural order.
template <int NW = 8>
__device__ __forceinline__ void dma_hc_row(const float2 *g, unsigned lds) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const char *src = reinterpret_cast<const char *>(g) + w * 1024 + lane * 16;
#pragma unroll
    for (int j = 0; j < 32 / NW; ++j) dma16(src + j * NW * 1024, lds + j * NW * 1024 + w * 1024);
}

// One antenna row for wave E of the pair.  On entry a/b hold the row's
// quarters E and E + 2; with PREF the first quarter of the next row is
// loaded into a at the row start (in flight through both transforms) and
// the second into b after the first MAC.  hr points at this row's Hc in LDS,
// DMA'd during the previous row; this row's first barrier publishes it
// (after vmcnt(0)) and the DMA of row r+1 (hnext, into LDS byte address
// hb_next) is issued right after that barrier, into the buffer every wave
// finished with in row r-1.  The second barrier: the partner has read the
// exchanged half from T before this wave's FFT transposes reuse it.
// Twiddles by recurrence from one per-lane base (hlds::tw_powers; 3-3.5 %
// faster here than 15 table reads per stage).
template <int E, bool PREF>
__device__ __forceinline__ void x_row(const float2 *__restrict__ next, const float2 *__restrict__ hr,
                                      int t, int pt, float2 *T, const float2 *Tp, const float2 *tw1,
                                      const float2 *tw2, pk::v2f wb0, pk::v2f wb1, float2 (&a)[16],
                                      float2 (&b)[16], float2 (&ae)[16], float2 (&ao)[16],
                                      const float2 *hnext, unsigned hb_next) {
    using namespace pk;
    v2f u[16], v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        u[m] = add(V(a[m]), V(b[m]));  // s
        v[m] = sub(V(a[m]), V(b[m]));  // d
    }
    float2 h[16];
    // wave 0 sends d and keeps s (= a); wave 1 sends s (= c) and keeps d:
    // 16-B pieces [m >> 1][t] (ds_write_b128 / ds_read_b128)
    float4 *T4 = reinterpret_cast<float4 *>(T);
    const float4 *Tp4 = reinterpret_cast<const float4 *>(Tp);
#pragma unroll
    for (int m = 0; m < 16; m += 2) {
        const float2 x0 = F(E ? u[m] : v[m]), x1 = F(E ? u[m + 1] : v[m + 1]);
        T4[(m >> 1) * 64 + t] = float4{x0.x, x0.y, x1.x, x1.y};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this row's Hc DMA landed
    td1024::lds_barrier();
    if (hnext) dma_hc_row(hnext, hb_next);
#pragma unroll
    for (int m = 0; m < 16; m += 2) {
        const float4 x = Tp4[(m >> 1) * 64 + t];
        if (E) {  // b
            u[m] = V(float2{x.x, x.y});
            u[m + 1] = V(float2{x.z, x.w});
        } else {  // c
            v[m] = V(float2{x.x, x.y});
            v[m + 1] = V(float2{x.z, x.w});
        }
    }
    td1024::lds_barrier();  // the partner has read T before the FFT reuses it
    // E = 0: u = a, v = c:  z0 = a + c, z2 = (a - c) W^(2 n0)
    // E = 1: u = b, v = d:  z1 = (b + (-i) d) W^(n0), z3 = (b - (-i) d) W^(3 n0)
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        v2f p, q;
        if (E) {
            p = add_mi(u[m], v[m]);
            q = sub_mi(u[m], v[m]);
        } else {
            p = add(u[m], v[m]);
            q = sub(u[m], v[m]);
        }
        u[m] = p;
        v[m] = q;
    }
#define OFDM_TWM(M)                                                                   \
    if (E) {                                                                          \
        u[M] = cmul(u[M], dif_tw<1, M>(wb0));                                         \
        v[M] = cmul(v[M], dif_tw<3, M>(wb1));                                         \
    } else {                                                                          \
        v[M] = cmul(v[M], dif_tw<2, M>(wb0));                                         \
    }
    OFDM_TWM(0) OFDM_TWM(1) OFDM_TWM(2) OFDM_TWM(3) OFDM_TWM(4) OFDM_TWM(5) OFDM_TWM(6)
    OFDM_TWM(7) OFDM_TWM(8) OFDM_TWM(9) OFDM_TWM(10) OFDM_TWM(11) OFDM_TWM(12) OFDM_TWM(13)
    OFDM_TWM(14) OFDM_TWM(15)
#undef OFDM_TWM
    float2 x[16];
    // Both FFT1024s of the row software-pipelined through the one transpose
    // image: A(u) -> write(u) -> read(u) issued -> A(v) computed while u's
    // transpose is in flight -> write(v), read(v) issued (LDS ops of a wave
    // complete in order, so v's writes follow u's reads) -> B(u) and MAC(u)
    // while v's transpose is in flight -> next row's loads -> B(v), MAC(v).
    v2f xu[16];
    if (PREF) row_load<true>(next + 1024 * E, t, a);  // in flight through both transforms
    // twiddle anchors read just in time, not held across the row
    // (hlds::tw_anchored; as row invariants they cost 37 spilled VGPRs):
    // stage A's with the LDS queue empty, stage B's behind v's transpose
    // reads, consumed after B's radix-16
    const hl::TwAnchors a_tw = hl::anchors_a(tw1, t);
    hl::fa_compute(u, a_tw);
    fa_write16(u, pt, T);
    fb_read16(t, T, xu);
    hl::fa_compute(v, a_tw);
    fa_write16(v, pt, T);
    fb_read16(t, T, u);  // u's registers are free: v's transpose lands in them
    __builtin_amdgcn_sched_barrier(0);
    const float4 *hr4 = reinterpret_cast<const float4 *>(hr);
#pragma unroll
    for (int k = 0; k < 16; k += 2) {  // plane 0, lands during B(u)
        const float4 x = hr4[(k >> 1) * 64 + t];
        h[k] = float2{x.x, x.y};
        h[k + 1] = float2{x.z, x.w};
    }
    hl::TwAnchors b_tw = hl::anchors_b(tw2, t);
    __builtin_amdgcn_sched_barrier(0);
    hl::fb_compute(xu, b_tw, t, x);
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // matrixMultThenSum (cpuLS.hpp:191-206), packed
        v2f a0 = V(ae[k]);
        pk::mac(a0, V(x[k]), V(h[k]));
        ae[k] = F(a0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 16; k += 2) {  // plane 1, lands during B(v)
        const float4 x = hr4[512 + (k >> 1) * 64 + t];
        h[k] = float2{x.x, x.y};
        h[k + 1] = float2{x.z, x.w};
    }
    __builtin_amdgcn_sched_barrier(0);
    if (PREF) row_load<true>(next + 1024 * (E + 2), t, b);
    b_tw = hl::anchors_b(tw2, t);
    hl::fb_compute(u, b_tw, t, x);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        v2f a0 = V(ao[k]);
        pk::mac(a0, V(x[k]), V(h[k]));
        ao[k] = F(a0);
    }
}

// ---------------------------------------------------------------------------
// MRC with the channel rows shared through LDS (k_mrc_td4096h): workgroup =
// 4 wave pairs = 4 consecutive data symbols of ONE frame (frame-aligned block
// map, bpf = ceil((S-1)/4) blocks per frame; tail pairs repeat the frame's
// last symbol without storing), so the frame's 32 KiB Hc row is fetched once
// per workgroup by LDS-DMA into a double buffer instead of by every wave
// from L2 (round 1's one-pair-per-workgroup kernel: Hc traffic = IQ
// traffic; a diagnostic without Hc loads ran 13 % faster).  The pairs' two exchange
// barriers per row become workgroup barriers and also publish the Hc row.
// LDS: tables 8 KiB + 8 transpose images 68 KiB + 2 x 32 KiB = 140 KiB, one
// workgroup (8 waves, 2 per SIMD as the 242-VGPR x kernel) per CU.
// ---------------------------------------------------------------------------
constexpr int H_PAIRS = 4;
constexpr size_t H_LDS = (size_t)(X_TAB + 2 * H_PAIRS * TS4 + 2 * C) * sizeof(float2);
static_assert(H_LDS <= 160 * 1024, "one workgroup per CU");

template <int E>
__device__ __forceinline__ void h_rows(const float2 *sym, int Cp, int R, const float2 *Hg, float2 *HB, int t,
                                       float2 *T, const float2 *Tp, const float2 *tw1, const float2 *tw2,
                                       pk::v2f wb0, pk::v2f wb1, float2 (&ae)[16], float2 (&ao)[16]) {
    float2 a[16], b[16];
    row_load<true>(sym + 1024 * E, t, a);
    row_load<true>(sym + 1024 * (E + 2), t, b);
    const unsigned hb0 = lds_addr(HB), hb1 = lds_addr(HB + C);
    const int pt = perm16(t);
    for (int r = 0; r + 1 < R; ++r)
        x_row<E, true>(sym + (long long)(r + 1) * Cp, HB + (r & 1) * C + E * 2048, t, pt, T, Tp, tw1, tw2, wb0, wb1, a,
                       b, ae, ao, Hg + (long long)(r + 1) * C, (r & 1) ? hb0 : hb1);
    x_row<E, false>(sym, HB + ((R - 1) & 1) * C + E * 2048, t, pt, T, Tp, tw1, tw2, wb0, wb1, a, b, ae, ao, nullptr, 0);
}

// The MRC of one logical block (H_PAIRS pairs = data symbols of frame f, pair
// `pair` on symbol j < nsym when `store`; s = its symbol slot) after the
// workgroup prologue: Hc row 0 DMA, tables, rows, normalise, staged stores.
__device__ __forceinline__ void mrc4096_block(const float2 *__restrict__ iq, int S, int R, int prefix,
                                              const float2 *Hc, const float *P, float2 *__restrict__ out,
                                              long long f, int j, bool store, int s, float2 *lds, int mode) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    const int e = w & 1, pair = w >> 1;
    const float2 *tw1 = lds, *tw2 = lds + hl::TW1S;
    float2 *T = lds + X_TAB + w * TS4;
    const float2 *Tp = lds + X_TAB + (w ^ 1) * TS4;
    float2 *HB = lds + X_TAB + 2 * H_PAIRS * TS4;  // [2][C] Hc rows
    const int nsym = S - 1;
    const float2 *Hg = Hc + f * (long long)R * C;
    dma_hc_row(Hg, lds_addr(HB));  // row 0; landed at the first row's barrier
    hl::fill(lds, lds + hl::TW1S);
    __syncthreads();

    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const pk::v2f wb0 = pk::V(g_tw[(e ? 1 : 2) * t]);
    const pk::v2f wb1 = pk::V(g_tw[3 * t]);
    float2 ae[16], ao[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) ae[k] = ao[k] = float2{0.f, 0.f};
    if (e)
        h_rows<1>(sym, Cp, R, Hg, HB, t, T, Tp, tw1, tw2, wb0, wb1, ae, ao);
    else
        h_rows<0>(sym, Cp, R, Hg, HB, t, T, Tp, tw1, tw2, wb0, wb1, ae, ao);
    const long long q = f * nsym + j;
    const int b0 = lane_bin0(t);
    float2 *o = out + q * K;
    const float *Pf = P + f * C;
    // Normalise, then stage the pair's 4095 outputs through its two transpose
    // images, 1024 positions per image and pass (pass h in image h & 1), and
    // store them as contiguous 512-B nontemporal wave stores: wave e stores
    // the image it owns.  Every wave (tail pairs too) takes part in the
    // workgroup barriers; only storing pairs write memory.
    if ((mode & 1) == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 4 * (b0 + 16 * k) + e;
            const float pe = Pf[be], po = Pf[be + 2];  // Pf[0] = 1: the DC slot
            // one reciprocal (v_rcp_f32) and two products per bin instead of
            // two IEEE divisions (within 2 ulp; frame_td.hip hlds_epilogue)
            const float re = __builtin_amdgcn_rcpf(pe), ro = __builtin_amdgcn_rcpf(po);
            ae[k] = float2{ae[k].x * re, ae[k].y * re};
            ao[k] = float2{ao[k].x * ro, ao[k].y * ro};
        }
    }
    float2 *Tpair = lds + X_TAB + 2 * pair * TS4;  // images of waves 2 pair, 2 pair + 1
    td1024::lds_barrier();  // both waves are done with their last transposes
#pragma unroll
    for (int h0 = 0; h0 < 4; h0 += 2) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int be = 4 * (b0 + 16 * k) + e;
            const int je = (mode & 1) ? be - 1 : out_pos(be - 1, K);  // be = 0: the DC bin, no output
            const int jo = (mode & 1) ? be + 1 : out_pos(be + 1, K);
            const int he = je >> 10, ho = jo >> 10;
            if (be > 0 && (he >> 1) == (h0 >> 1))
                Tpair[(he & 1) * TS4 + ((je & 1023) >> 6) * TP4 + (je & 63)] = ae[k];
            if ((ho >> 1) == (h0 >> 1)) Tpair[(ho & 1) * TS4 + ((jo & 1023) >> 6) * TP4 + (jo & 63)] = ao[k];
        }
        td1024::lds_barrier();
        if (store) {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int jj = 1024 * (h0 + e) + t + 64 * m;
                if (jj < K)
                    __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, T[m * TP4 + t]),
                                                reinterpret_cast<unsigned long long *>(o + jj));
            }
        }
        td1024::lds_barrier();
    }
}

__global__ void __attribute__((amdgpu_flat_work_group_size(128 * H_PAIRS, 128 * H_PAIRS), amdgpu_waves_per_eu(2, 2)))
k_mrc_td4096h(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
              const float *__restrict__ P, float2 *__restrict__ out, long long nframes, long long nblocks,
              Tickets tk, long long k0, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int pair = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);
    OFDM_DIAG_BEGIN()
    // the logical block is a work ticket (wave_fft1024.hpp take_block: own
    // XCD's range of consecutive blocks first -- a frame's blocks share an
    // L2 -- then the others'); the slot is wave 0's transpose image, first
    // written after mrc4096_block's table barrier
    const long long lb = wg_take_block(tk, nblocks, k0, blockIdx.x, reinterpret_cast<long long *>(lds + X_TAB));
    if (lb < 0) return;  // whole workgroup: every block taken
    const int nsym = S - 1;
    const long long bpf = (nsym + H_PAIRS - 1) / H_PAIRS;
    const long long f = lb / bpf;
    const int j = (int)(lb - f * bpf) * H_PAIRS + pair;  // data symbol index within the frame
    const bool store = j < nsym;
    const int s = 1 + (store ? j : nsym - 1);
    mrc4096_block(iq, S, R, prefix, Hc, P, out, f, j, store, s, lds, mode);
    OFDM_DIAG_END(td4096);
}


}  // namespace td4096

hipError_t launch_ls_td4096(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial, hipStream_t s) {
    using namespace td4096;
    if (nframes <= 0) return hipSuccess;
    if (nframes > 0x7fffffffll) return hipErrorInvalidValue;
    auto kern = k_ls_td4096<LS_WAVES>;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)ls_lds(LS_WAVES)); e != hipSuccess)
        return e;  // > 64 KiB of dynamic LDS
    hipLaunchKernelGGL(kern, dim3((unsigned)nframes), dim3(64 * LS_WAVES), ls_lds(LS_WAVES), s, iq, S, R,
                       prefix, X, Hc, P, partial);
    return hipGetLastError();
}

hipError_t launch_mrc_td4096(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode, Tickets tk,
                             hipStream_t s) {
    using namespace td4096;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    const long long bpf = ((S - 1) + H_PAIRS - 1) / H_PAIRS, nb = nframes * bpf, g = td1024::ticket_grid(nb);
    if (g > 0x7fffffffll) return hipErrorInvalidValue;
    // The row's two FFT1024s software-pipelined through the transpose
    // image and the first quarter of the next row issued at the row start
    // (same-process A/B, R=32 x 300 frames: 6.81 vs 7.53 ms, bit-identical;
    // profiles/r3/r3_ab_il*_c4096.jsonl)
    auto kern = k_mrc_td4096h;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)H_LDS); e != hipSuccess)
        return e;  // > 64 KiB of dynamic LDS
    hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(128 * H_PAIRS), H_LDS, s, iq, S, R, prefix, Hc, P, out, nframes,
                       nb, tk, td1024::ticket_k0(1), mode);
    return hipGetLastError();
}


}  // namespace ofdm
