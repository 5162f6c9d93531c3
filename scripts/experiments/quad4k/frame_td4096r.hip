// frame_td4096r.hip -- fused time-domain receiver for C = 4096 on wave QUADS
// with the register-only FFT (rfft1024.hpp) and LDS-DMA row prefetch.
//
// A data symbol's 4096-point row is shared by four waves.  Wave c (0..3) of
// the quad computes the bins 4 k + c by one radix-4 decimation-in-frequency
// step (n = n0 + 1024 n1):
//   z_c[n0] = sum_n1 x[n0 + 1024 n1] (-i)^(c n1) W4096^(c n0),
//   X[4 k + c] = FFT1024(z_c)[k]
// so each wave holds 16 bins per lane and 16 accumulators: the register
// state of the C = 1024 receiver, 4 waves per SIMD (k_mrc_td4096h, a wave
// PAIR per symbol with 32 bins per lane, runs at 2).  The FFT needs no
// transpose image, which leaves the LDS to the rows themselves: the quad's
// next 32 KiB row is DMA'd (global_load_lds_dwordx4, no registers) into the
// quad's row buffer while the current row is transformed, and each wave
// reads its four quarters from there.
//
// Workgroup = 4 quads = 4 consecutive data symbols of ONE frame (frame-aligned
// block map, ceil((S-1)/4) blocks per frame; tail quads repeat the frame's
// last symbol without storing), 16 waves, one per CU.  LDS: 4 row buffers
// (128 KiB) + the W1024^(t k2) table (7.5 KiB).  Per antenna row two
// workgroup barriers: B1 (the row has landed: every wave waited for its own
// DMA pieces), B2 (every wave has read the row: the next row's DMA may
// overwrite it).  Hc for the wave's 16 bins comes from L2 (8 dwordx4 per
// lane, issued before the next row's DMA and waited for by an explicit
// vmcnt so the wait does not drain the DMA).
//
// A/B build only (OFDM_AB_KNOBS; switch MRC4K_R=1): correct and tested, but
// 21 % slower than k_mrc_td4096h (profiles/r2_ab/quad4k_ab.jsonl).
//
// Hc layout (LS kernel below; stages.hip hc_pos): per (frame, antenna) four
// planes c of 512 float4, float4 i*64 + t = (Hc[4 b(t, 2i) + c],
// Hc[4 b(t, 2i+1) + c]), b(t, j) = rfft_bin(t, j).  P bin-indexed [F][C].
#ifdef OFDM_AB_KNOBS
#include "launch.hpp"
#include "rfft1024.hpp"

namespace ofdm {
namespace td4096r {

using pk::v2f;
typedef float v4f __attribute__((ext_vector_type(4)));
using td1024::dma16;
using td1024::lds_addr;
using td1024::row_load;
namespace hl = td1024::hlds;

constexpr int C = 4096;
constexpr int K = C - 1;
constexpr int QUADS = 4;
constexpr int WAVES = 4 * QUADS;
// NQ quads per workgroup: NQ row buffers + the Hc row (+ the W1024^(t k2)
// table when it fits: NQ = 3)
constexpr bool tab(int nq) { return nq < 4; }
constexpr int CTAB = 6 * 64;  // per-lane FFT constants [6][64] float2, then W4096^(c t) [4][64] (tab(NQ) only)
constexpr size_t lds_bytes(int nq) {
    return (size_t)(nq + 1) * C * sizeof(float2) + (tab(nq) ? (size_t)(hl::TW1S + CTAB + 256) * sizeof(float2) : 0);
}
// the lane constants of rfft::make_consts from w1 = W64^(t & 15) and W1024^t
// alone (per row, a few VALU; only two complex registers held across the
// loop): W16^(t_lo & 7) = (-1)^b3 w1^4, W8^(t_lo & 3) = (-1)^b2 w1^8
__device__ __forceinline__ rfft::Consts derive_consts(v2f w1024, v2f w1, int t) {
    rfft::Consts k;
    k.w1024 = w1024;
    k.w1 = w1;
    k.w2 = pk::cmul(w1, w1);
    k.w3 = pk::cmul(k.w2, w1);
    const v2f w4 = pk::cmul(k.w2, k.w2), w8 = pk::cmul(w4, w4);
    const bool b3 = (t >> 3) & 1, b2 = (t >> 2) & 1;
    k.c1 = b3 ? w4 : (v2f){1.f, 0.f};  // -W16^(t_lo & 7) = w4 when b3
    const float g = td1024::quad_g(t & 3);
    k.c2 = b2 ? (v2f){-g * w8.x, -g * w8.y} : (v2f){g, 0.f};
    k.s1 = b3 ? -1.f : 1.f;
    return k;
}

// the lane constants of rfft::make_consts from LDS (row loop: no registers
// held across the loop, no vector-memory load the DMA accounting would see)
__device__ __forceinline__ rfft::Consts lds_consts(const float2 *ct, int t) {
    rfft::Consts k;
    k.w1024 = pk::V(ct[t]);
    k.w1 = pk::V(ct[64 + t]);
    k.w2 = pk::V(ct[128 + t]);
    k.w3 = pk::V(ct[192 + t]);
    k.c1 = pk::V(ct[256 + t]);
    k.c2 = pk::V(ct[320 + t]);
    k.s1 = (t & 8) ? -1.f : 1.f;
    return k;
}
static_assert(lds_bytes(4) == 160 * 1024 && lds_bytes(3) <= 160 * 1024, "one workgroup per CU");

template <int CC, int M>
__device__ __forceinline__ v2f dif_tw(v2f base) {  // base * W64^(CC * M)
    if constexpr ((CC * M) % 64 == 0) return base;
    constexpr float2 w = tw_const<64, CC * M>();
    return pk::cmul_s_v(base, (v2f){w.x, w.y});
}

// z_CC[m] from the four quarters x_n1[m] = q[1024 n1 + t + 64 m] (LDS or
// global), times W4096^(CC n0) = wb W64^(CC m)
template <int CC, typename Src>
__device__ __forceinline__ void combine(Src q, int t, v2f wb, float2 (&z)[16]) {
#define OFDM_CMB(M)                                                                        \
    {                                                                                      \
        const v2f x0 = pk::V(q[(M) * 64 + t]), x1 = pk::V(q[1024 + (M) * 64 + t]);         \
        const v2f x2 = pk::V(q[2048 + (M) * 64 + t]), x3 = pk::V(q[3072 + (M) * 64 + t]);  \
        v2f r;                                                                             \
        if constexpr (CC == 0) r = pk::add(pk::add(x0, x2), pk::add(x1, x3));              \
        if constexpr (CC == 2) r = pk::sub(pk::add(x0, x2), pk::add(x1, x3));              \
        if constexpr (CC == 1) r = pk::add_mi(pk::sub(x0, x2), pk::sub(x1, x3));           \
        if constexpr (CC == 3) r = pk::sub_mi(pk::sub(x0, x2), pk::sub(x1, x3));           \
        if constexpr (CC != 0) r = pk::cmul(r, dif_tw<CC, M>(wb));                         \
        z[M] = pk::F(r);                                                                   \
    }
    // two m at a time: the scheduler would otherwise issue all 64 reads first
#define OFDM_SB __builtin_amdgcn_sched_barrier(0);
    OFDM_CMB(0) OFDM_CMB(1) OFDM_SB OFDM_CMB(2) OFDM_CMB(3) OFDM_SB OFDM_CMB(4) OFDM_CMB(5) OFDM_SB
    OFDM_CMB(6) OFDM_CMB(7) OFDM_SB OFDM_CMB(8) OFDM_CMB(9) OFDM_SB OFDM_CMB(10) OFDM_CMB(11) OFDM_SB
    OFDM_CMB(12) OFDM_CMB(13) OFDM_SB OFDM_CMB(14) OFDM_CMB(15)
#undef OFDM_SB
#undef OFDM_CMB
}

// N pieces of 1 KiB (16 B per lane) from global memory into LDS, STRIDE
// bytes apart on both sides: one address register pair advanced in the asm
// (the compiler would otherwise keep N 64-bit addresses live) and M0 stepped
// by s_add_u32; SCC, which those adds change behind the compiler's back, is
// saved first and restored last (s_cselect / s_cmp); M0 saved/restored;
// s_nop for the M0 -> LDS-DMA hazard.  No "memory" clobber (it makes the
// compiler keep far more registers live across the FFT): the LDS the DMA
// writes is ordered against its readers by the explicit vmcnt waits and the
// workgroup barriers (asm with "memory" clobbers) alone.
template <int N, int STRIDE>
__device__ __forceinline__ void dma_pieces(const void *g, unsigned lds) {
    static_assert(N == 8 || N == 2, "8 or 2 pieces");
    unsigned keep, scc;
    const void *a = g;
#define OFDM_P "s_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
#define OFDM_S "v_lshl_add_u64 %2, %2, 0, %4\n\ts_add_u32 m0, m0, %5\n\t"
#define OFDM_HEAD "s_cselect_b32 %1, -1, 0\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\t"
#define OFDM_TAIL "s_mov_b32 m0, %0\n\ts_cmp_lg_u32 %1, 0"
    if constexpr (N == 8)
        asm volatile(OFDM_HEAD OFDM_P OFDM_S OFDM_P OFDM_S OFDM_P OFDM_S OFDM_P OFDM_S OFDM_P OFDM_S OFDM_P OFDM_S
                         OFDM_P OFDM_S OFDM_P OFDM_TAIL
                     : "=&s"(keep), "=&s"(scc), "+v"(a)
                     : "s"(lds), "s"((unsigned long long)STRIDE), "n"(STRIDE));
    else
        asm volatile(OFDM_HEAD OFDM_P OFDM_S OFDM_P OFDM_TAIL
                     : "=&s"(keep), "=&s"(scc), "+v"(a)
                     : "s"(lds), "s"((unsigned long long)STRIDE), "n"(STRIDE));
#undef OFDM_P
#undef OFDM_S
#undef OFDM_HEAD
#undef OFDM_TAIL
}

// the quad's 32 KiB row into its buffer: wave c moves the 1 KiB pieces c,
// c + 4, ..., c + 28
__device__ __forceinline__ void dma_row(const float2 *row, unsigned rb, int c, int lane) {
    dma_pieces<8, 4096>(reinterpret_cast<const char *>(row) + c * 1024 + lane * 16, rb + c * 1024);
}

// Hc row r of the frame into HB by the whole workgroup (4 NQ waves): wave w
// moves the 1 KiB pieces w, w + 16 (NQ = 4) or w, w + 12, w + 24 (NQ = 3)
template <int NQ>
__device__ __forceinline__ void dma_hc(const float2 *hrow, unsigned hb, int w, int lane) {
    const char *src = reinterpret_cast<const char *>(hrow) + lane * 16;
    if constexpr (NQ == 4) {
        dma_pieces<2, 16384>(src + w * 1024, hb + w * 1024);
    } else {
#pragma unroll
        for (int p = 0; p < 32; p += 4 * NQ)
            if (p + w < 32) dma16(src + (p + w) * 1024, hb + (p + w) * 1024);
    }
}

// One antenna row of wave CC of a quad.  PF: the next row's DMA is issued
// after B2 (every row but the last; the last is peeled so that the row body
// has no branch: a conditional asm statement in front of the FFT makes the
// compiler spill the accumulators).
template <int CC, int NQ, bool PF>
__device__ __forceinline__ void quad_row(const float2 *next, const float2 *hrow, v2f w1024, v2f w64, v2f wb0,
                                         int w, const float2 *rbq, unsigned rb, const float4 *HB4, unsigned hb,
                                         const float2 *tw1, float2 (&acc)[16]) {
    int t = __lane_id();  // recomputed per row (v_mbcnt): nothing lane-derived held across the loop
    asm volatile("" : "+v"(t));
    v2f wb = wb0;
    rfft::Consts k;
    if constexpr (tab(NQ)) {
        k = lds_consts(tw1 + hl::TW1S, t);
        wb = pk::V(tw1[hl::TW1S + CTAB + CC * 64 + t]);
    } else {
        k = derive_consts(w1024, w64, t);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of this row
    td1024::lds_barrier();  // B1: the row is complete; every wave is past the previous MAC
    float2 z[16];
    combine<CC>(rbq, t, wb, z);
    td1024::lds_barrier();  // B2: every wave has read its quarters of the row
    dma_hc<NQ>(hrow, hb, w, t);
    if constexpr (PF) dma_row(next, rb, CC, t);
    rfft::fft1024<!tab(NQ)>(z, t, tw1, k);
    if constexpr (PF)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // own Hc pieces (older than the row's 8)
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    td1024::lds_barrier();  // B3: the Hc row is complete
    const float4 *hp = HB4 + CC * 512 + t;
    // matrixMultThenSum (cpuLS.hpp:203-204), antennas in order
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i & 1) __builtin_amdgcn_sched_barrier(0);
        const float4 h = hp[i * 64];
        v2f a0 = pk::V(acc[2 * i]), a1 = pk::V(acc[2 * i + 1]);
        pk::mac(a0, pk::V(z[2 * i]), (v2f){h.x, h.y});
        pk::mac(a1, pk::V(z[2 * i + 1]), (v2f){h.z, h.w});
        acc[2 * i] = pk::F(a0);
        acc[2 * i + 1] = pk::F(a1);
    }
}

template <int CC, int NQ, int DBG = 0>
__device__ __forceinline__ void quad_rows(const float2 *sym, int Cp, int R, const float2 *Hg, int t0, int w,
                                          const float2 *rbq, unsigned rb, const float4 *HB4, unsigned hb,
                                          const float2 *tw1, float2 (&acc)[16]) {
    const v2f w1024 = pk::V(g_tw[t0 * (OFDM_TW_N / 1024)]), w64 = pk::V(g_tw[(t0 & 15) * (OFDM_TW_N / 64)]);
    const v2f wb0 = pk::V(g_tw[(CC * t0) * (OFDM_TW_N / C)]);  // W4096^(CC t)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = float2{0.f, 0.f};
    for (int r = 0; r + 1 < R; ++r) {
        if constexpr ((DBG & 64) != 0)  // diagnostic: no row DMA after row 0 (compute only)
            quad_row<CC, NQ, false>(nullptr, Hg + (long long)r * C, w1024, w64, wb0, w, rbq, rb, HB4, hb, tw1, acc);
        else
            quad_row<CC, NQ, true>(sym + (long long)(r + 1) * Cp, Hg + (long long)r * C, w1024, w64, wb0, w, rbq,
                                   rb, HB4, hb, tw1, acc);
    }
    quad_row<CC, NQ, false>(nullptr, Hg + (long long)(R - 1) * C, w1024, w64, wb0, w, rbq, rb, HB4, hb, tw1, acc);
}

// DBG (A/B build only, wrong results by design): bit 6 no DMA after row 0
// (compute only).
template <int NQ, int DBG = 0>
__global__ void __attribute__((amdgpu_flat_work_group_size(256 * NQ, 256 * NQ), amdgpu_waves_per_eu(NQ, NQ)))
k_mrc_td4096r(const float2 *__restrict__ iq, int S, int R, int prefix, const float2 *__restrict__ Hc,
              const float *__restrict__ P, float2 *__restrict__ out, long long nblocks, long long per_xcd,
              int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t = threadIdx.x & 63;
    const int c = w & 3, quad = w >> 2;
    float2 *rbq = lds + quad * C;
    float4 *HB4 = reinterpret_cast<float4 *>(lds + NQ * C);  // the frame's Hc row
    float2 *tw1 = lds + (NQ + 1) * C;                         // tab(NQ): W1024^(t k2), [k2 - 1][t]
    const long long pb = blockIdx.x;
    const long long lb = (pb & 7) * per_xcd + (pb >> 3);  // XCD-grouped: a frame's blocks share an L2
    if (lb >= nblocks) return;                            // whole workgroup
    const int nsym = S - 1;
    const long long bpf = (nsym + NQ - 1) / NQ;
    const long long f = lb / bpf;
    const int j = (int)(lb - f * bpf) * NQ + quad;  // data symbol index within the frame
    const bool store = j < nsym;
    const int s = 1 + (store ? j : nsym - 1);
    const int Cp = C + prefix;
    const float2 *sym = iq + (f * S + s) * (long long)R * Cp + prefix;
    const unsigned rb = lds_addr(rbq);
    dma_row(sym, rb, c, t);  // row 0
    if constexpr (tab(NQ)) {
        for (int i = threadIdx.x; i < hl::TW1S; i += blockDim.x) {
            const int k2 = 1 + i / 64, tt = i % 64;
            tw1[i] = g_tw[((tt * k2) & 1023) * (OFDM_TW_N / 1024)];
        }
        if (threadIdx.x < 64) {  // lane constants + W4096^(c t) for c = 0..3
            const rfft::Consts k = rfft::make_consts(t);
            float2 *ct = tw1 + hl::TW1S;
            ct[t] = pk::F(k.w1024);
            ct[64 + t] = pk::F(k.w1);
            ct[128 + t] = pk::F(k.w2);
            ct[192 + t] = pk::F(k.w3);
            ct[256 + t] = pk::F(k.c1);
            ct[320 + t] = pk::F(k.c2);
            for (int cc = 0; cc < 4; ++cc) ct[CTAB + cc * 64 + t] = g_tw[(cc * t) * (OFDM_TW_N / C)];
        }
    }
    const float2 *Hg = Hc + f * (long long)R * C;
    const unsigned hb = lds_addr(HB4);
    float2 acc[16];
    if (c == 0) quad_rows<0, NQ, DBG>(sym, Cp, R, Hg, t, w, rbq, rb, HB4, hb, tw1, acc);
    else if (c == 1) quad_rows<1, NQ, DBG>(sym, Cp, R, Hg, t, w, rbq, rb, HB4, hb, tw1, acc);
    else if (c == 2) quad_rows<2, NQ, DBG>(sym, Cp, R, Hg, t, w, rbq, rb, HB4, hb, tw1, acc);
    else quad_rows<3, NQ, DBG>(sym, Cp, R, Hg, t, w, rbq, rb, HB4, hb, tw1, acc);

    // normalise, stage the quad's 4095 outputs at their rotated positions in
    // its row buffer (free after the last B2), store: wave c writes positions
    // [1024 c, 1024 c + 1024) as 16 contiguous 512-B nontemporal wave stores
    int tl = t;
    asm volatile("" : "+v"(tl));  // keep the epilogue's index arithmetic below the row loop
    const float *Pf = P + f * C;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        const int b = 4 * rfft::rfft_bin(tl, jj) + c;
        if (b == 0) continue;  // the DC bin: no output
        float2 v = acc[jj];
        int pos = b - 1;
        if ((mode & 1) == 0) {
            const float pv = Pf[b];
            v = float2{v.x / pv, v.y / pv};
            pos = out_pos(b - 1, K);
        }
        rbq[pos] = v;
    }
    td1024::lds_barrier();
    if (!store) return;
    float2 *o = out + (f * nsym + j) * (long long)K;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int jj = 1024 * c + tl + 64 * m;
        if (jj < K)
            __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, rbq[jj]),
                                        reinterpret_cast<unsigned long long *>(o + jj));
    }
}

// ---------------------------------------------------------------------------
// LS: one workgroup (4 quads) per frame; quad q takes antenna rows q, q + 4,
// ...; wave c reads the four quarters of its row straight from memory.
// Pilots in LDS; partial |H|^2 per quad combined in quad order.
// ---------------------------------------------------------------------------
constexpr size_t LS_LDS = (size_t)hl::TW1S * sizeof(float2) + (size_t)C * sizeof(float2) +
                          (size_t)QUADS * C * sizeof(float);

template <int CC>
__device__ __forceinline__ void ls_rows(const float2 *pilot, int Cp, int R, int q, int t, const float2 *tw1,
                                        const float2 *xs, float4 *Hf, float *pp) {
    const rfft::Consts k = rfft::make_consts(t);
    const v2f wb = pk::V(g_tw[(CC * t) * (OFDM_TW_N / C)]);
    float p[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) p[j] = 0.f;
    for (int r = q; r < R; r += QUADS) {
        float2 z[16];
        combine<CC>(pilot + (long long)r * Cp, t, wb, z);
        rfft::fft1024(z, t, tw1, k);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int b = 4 * rfft::rfft_bin(t, j) + CC;
            // divideOneRow + conj (cpuLS.hpp:233-244, 303-307); DC bin dropped
            float2 h = ls_conj(z[j], xs[b]);
            if (b == 0) h = float2{0.f, 0.f};
            p[j] = p[j] + (h.x * h.x) + (h.y * h.y);  // findDistSqrd order within the quad
            z[j] = h;
        }
        td1024::hc_store(Hf + (long long)r * (C / 2) + CC * 512, t, z);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) pp[q * C + 4 * rfft::rfft_bin(t, j) + CC] = p[j];
}

__global__ void __launch_bounds__(1024) k_ls_td4096r(const float2 *__restrict__ iq, int S, int R, int prefix,
                                                     const float2 *__restrict__ X, float2 *__restrict__ Hc,
                                                     float *__restrict__ P, int partial) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    const int c = w & 3, q = w >> 2;
    float2 *tw1 = lds;
    float2 *xs = lds + hl::TW1S;                          // xs[b] = X[b - 1], xs[0] unused
    float *pp = reinterpret_cast<float *>(xs + C);        // [QUADS][C]
    for (int i = threadIdx.x; i < hl::TW1S; i += blockDim.x) {
        const int k2 = 1 + i / 64, tt = i % 64;
        tw1[i] = g_tw[((tt * k2) & 1023) * (OFDM_TW_N / 1024)];
    }
    for (int b = threadIdx.x; b < C; b += blockDim.x) xs[b] = b ? X[b - 1] : float2{1.f, 0.f};
    for (int i = threadIdx.x; i < QUADS * C; i += blockDim.x) pp[i] = 0.f;  // quads without rows (R < 4)
    __syncthreads();
    const long long f = blockIdx.x;
    const int Cp = C + prefix;
    const float2 *pilot = iq + f * (long long)S * R * Cp + prefix;
    float4 *Hf = reinterpret_cast<float4 *>(Hc + f * (long long)R * C);
    if (c == 0) ls_rows<0>(pilot, Cp, R, q, t, tw1, xs, Hf, pp);
    else if (c == 1) ls_rows<1>(pilot, Cp, R, q, t, tw1, xs, Hf, pp);
    else if (c == 2) ls_rows<2>(pilot, Cp, R, q, t, tw1, xs, Hf, pp);
    else ls_rows<3>(pilot, Cp, R, q, t, tw1, xs, Hf, pp);
    __syncthreads();
    float *Pf = P + f * C;
    for (int b = threadIdx.x; b < C; b += blockDim.x) {
        float sum = pp[b];
        for (int i = 1; i < QUADS; ++i) sum = sum + pp[i * C + b];  // antennas in quad order
        Pf[b] = b == 0 ? (partial ? 0.f : 1.f) : sum;
    }
}

}  // namespace td4096r

// Rows must be 16-byte aligned for the row DMA: iq 16-B aligned, prefix even.
bool td4096r_ok(const float2 *iq, int prefix) {
    return ab_knob("MRC4K_R", 0) && (reinterpret_cast<uintptr_t>(iq) & 15) == 0 && (prefix & 1) == 0;
}

hipError_t launch_ls_td4096r(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *X,
                             float2 *Hc, float *P, int partial, hipStream_t s) {
    using namespace td4096r;
    if (nframes <= 0) return hipSuccess;
    if (nframes > 0x7fffffffll) return hipErrorInvalidValue;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(k_ls_td4096r), (int)LS_LDS); e != hipSuccess)
        return e;
    hipLaunchKernelGGL(k_ls_td4096r, dim3((unsigned)nframes), dim3(64 * WAVES), LS_LDS, s, iq, S, R, prefix, X,
                       Hc, P, partial);
    return hipGetLastError();
}

hipError_t launch_mrc_td4096r(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hc,
                              const float *P, float2 *out, int mode, hipStream_t s) {
    using namespace td4096r;
    const long long nq = nframes * (S - 1);
    if (nq <= 0) return hipSuccess;
    auto go = [&](auto kern, int nq) {
        const long long bpf = ((S - 1) + nq - 1) / nq, nb = nframes * bpf, pxcd = (nb + 7) / 8;
        if (pxcd * 8 > 0x7fffffffll) return hipErrorInvalidValue;
        const size_t lds = lds_bytes(nq);
        if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)lds); e != hipSuccess) return e;
        hipLaunchKernelGGL(kern, dim3((unsigned)(pxcd * 8)), dim3(256 * nq), lds, s, iq, S, R, prefix, Hc, P, out,
                           nb, pxcd, mode);
        return hipGetLastError();
    };
#ifdef OFDM_AB_KNOBS
    const int v = ab_knob("MRC4K_R", 1);
    if (v == 64 + 3) return go(k_mrc_td4096r<3, 64>, 3);  // diagnostics: no row DMA after row 0
    if (v == 64 + 4) return go(k_mrc_td4096r<4, 64>, 4);
    if (v == 3) return go(k_mrc_td4096r<3>, 3);  // 3 quads (3 waves/SIMD, the twiddle table in LDS)
#endif
    return go(k_mrc_td4096r<4>, 4);
}

}  // namespace ofdm
#endif  // OFDM_AB_KNOBS
