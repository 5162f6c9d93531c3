// wave_fft1024.hpp -- 1024-point forward FFT on one 64-lane wave (CDNA4),
// shared by the fused receiver kernels (frame_td.hip, frame_td2048.hip).
//
// Four-step, N = 64 x 16: lane t holds x[t + 64 m], m < 16.
//   A[t][k2]  = FFT16_m(x[t + 64 m]) * W1024^(t k2)                 k2 < 16
//   X[k2 + 16 k1] = DFT64_t(A[t][k2])                                k1 < 64
// The 64-point DFTs run on lane quads after an LDS transpose: lane
// t = 4 q + a (q = k2, a < 4) holds A[a + 4 l'][q], l' < 16, and
//   B_a[k'] = FFT16_l'(A[a + 4 l'][q]) * W64^(a k')                   k' < 16
//   X[q + 16 (k' + 16 c)] = sum_a B_a[k'] W4^(a c)                    c < 4
// the last sum being a radix-2 x 2 exchange inside the quad (DPP).  Lane
// (q, a) finally owns bins b = q + 256 c(a) + 16 k', c(a) = (a >> 1) + 2 (a & 1).
#pragma once
#include "common.hpp"
#include "launch.hpp"
#include "pk.hpp"

namespace ofdm {
namespace td1024 {

constexpr int C = 1024;
constexpr int K = C - 1;
constexpr int TP = 68;              // pitch of the [16][64] transpose image (conflict free)
constexpr int TBUF = 16 * TP;       // float2 per wave
constexpr int TW1P = 17;            // pitch of TW1[t][k2] = W1024^(t k2)
constexpr int TW1BUF = 64 * TW1P;
constexpr int TW2P = 17;            // pitch of TW2[a][k'] = g(a) W64^(a k'): 4 rows on 4 banks
constexpr int TW2BUF = 4 * TW2P;
constexpr int TWBUF = TW1BUF + TW2BUF;

__device__ __forceinline__ void wave_lds_sync() {
    // LDS operations of one wave execute in order; this only stops the
    // compiler from moving LDS accesses across the exchange point.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier that orders LDS only: unlike __syncthreads() it does not
// make the compiler drain outstanding global loads (vmcnt), so a prefetched
// row stays in flight across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

typedef __attribute__((address_space(3))) void lvoid_t;
__device__ __forceinline__ unsigned lds_addr(const void *p) { return (unsigned)(size_t)(lvoid_t *)p; }

// 16 B per lane straight into LDS at byte lds + 16 lane (global_load_lds_dwordx4
// in inline asm: the builtin makes the compiler wait vmcnt(0) before every LDS
// read; M0 saved/restored in the same statement, s_nop for the M0 hazard).
__device__ __forceinline__ void dma16(const void *g, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}

// Quad-DFT signs (found by exhaustive search, verified in tests): lane a of a
// quad pre-scales its B_a by g(a) (folded into TW2) so that both radix-2
// stages are one fma(dpp(x), S, x) per float with exact results:
//   g = (1,-1,-1,1), S1 = (-1,-1,1,1) [partner a^2], S2 = (-1,1,-1,1) [a^1],
//   lane 3 multiplies by -i between the stages.
__device__ __forceinline__ float quad_g(int a) { return (a == 0 || a == 3) ? 1.f : -1.f; }

__device__ __forceinline__ void fill_twiddles(float2 *tw) {
    for (int i = threadIdx.x; i < TW1BUF; i += blockDim.x) {
        const int t = i / TW1P, k2 = i % TW1P;
        tw[i] = k2 < 16 ? g_tw[((t * k2) & (C - 1)) * (OFDM_TW_N / C)] : float2{0.f, 0.f};
    }
    for (int i = threadIdx.x; i < TW2BUF; i += blockDim.x) {
        const int a = i / TW2P, k = i % TW2P;
        const float2 w = g_tw[((16 * a * k) & (C - 1)) * (OFDM_TW_N / C)];
        const float g = quad_g(a);
        tw[TW1BUF + i] = k < 16 ? float2{g * w.x, g * w.y} : float2{0.f, 0.f};
    }
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL,
                                                              0xF, 0xF, true));
}
constexpr int DPP_XOR1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;  // quad_perm [2,3,0,1]

// a[m] = src[t + 64 m]: 16 coalesced 512-byte wave loads.  NT: non-temporal
// (streamed once; keeps L2 for the per-frame channel estimates).
template <bool NT = false>
__device__ __forceinline__ void row_load(const float2 *__restrict__ src, int t, float2 (&a)[16]) {
    if (NT) {
        const unsigned long long *p = reinterpret_cast<const unsigned long long *>(src) + t;
#pragma unroll
        for (int m = 0; m < 16; ++m)
            a[m] = __builtin_bit_cast(float2, __builtin_nontemporal_load(p + 64 * m));
    } else {
#pragma unroll
        for (int m = 0; m < 16; ++m) a[m] = src[t + 64 * m];
    }
}

// v[k] = dpp(v[k]) * S + v[k] for 16 floats, one v_fmac_f32_dpp each (the
// compiler would emit v_mov_dpp + fma + an s_nop per value).  The leading
// s_nop 1 covers the "VALU writes VGPR -> DPP reads it" hazard (2 wait states)
// for whatever the compiler computed last; inside the block no instruction
// reads another's output (cdna_hip_programming.md 5.7).
#define OFDM_DPP_Q(CTRL) "quad_perm:" CTRL " row_mask:0xf bank_mask:0xf"
template <int CTRL>
__device__ __forceinline__ void quad_fmac_dpp(float (&v)[16], float S) {
#define OFDM_F(i) "v_fmac_f32_dpp %" #i ", %" #i ", %16 " OFDM_DPP_Q(QP) "\n\t"
    if constexpr (CTRL == 0x4E) {
#define QP "[2,3,0,1]"
        asm("s_nop 1\n\t" OFDM_F(0) OFDM_F(1) OFDM_F(2) OFDM_F(3) OFDM_F(4) OFDM_F(5) OFDM_F(6)
                OFDM_F(7) OFDM_F(8) OFDM_F(9) OFDM_F(10) OFDM_F(11) OFDM_F(12) OFDM_F(13) OFDM_F(14)
                    OFDM_F(15)
            : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
              "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]),
              "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
            : "v"(S));
#undef QP
    } else {
        static_assert(CTRL == 0xB1, "quad xor 1 or xor 2");
#define QP "[1,0,3,2]"
        asm("s_nop 1\n\t" OFDM_F(0) OFDM_F(1) OFDM_F(2) OFDM_F(3) OFDM_F(4) OFDM_F(5) OFDM_F(6)
                OFDM_F(7) OFDM_F(8) OFDM_F(9) OFDM_F(10) OFDM_F(11) OFDM_F(12) OFDM_F(13) OFDM_F(14)
                    OFDM_F(15)
            : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
              "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]),
              "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
            : "v"(S));
#undef QP
    }
#undef OFDM_F
}
#undef OFDM_DPP_Q

// 4-point DFT over the lanes of each quad (see header), in place.
__device__ __forceinline__ void quad_dft(float2 (&x)[16], int qa) {
    // two radix-2 stages, one fma per float each
    const float S1 = (qa & 2) ? 1.f : -1.f;
    const float S2 = (qa & 1) ? 1.f : -1.f;
    // lanes with qa == 3 multiply by -i between the stages: (x, y) -> (y, -x)
    const unsigned long long rot = __builtin_amdgcn_ballot_w64(qa == 3);
    float xr[16], xi[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { xr[k] = x[k].x; xi[k] = x[k].y; }
    quad_fmac_dpp<DPP_XOR2>(xr, S1);
    quad_fmac_dpp<DPP_XOR2>(xi, S1);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        float nx;
        asm("v_cndmask_b32_e64 %0, %2, %3, %4\n\tv_cndmask_b32_e64 %1, %3, -%2, %4"
            : "=&v"(nx), "=v"(xi[k])
            : "v"(xr[k]), "v"(xi[k]), "s"(rot));
        xr[k] = nx;
    }
    quad_fmac_dpp<DPP_XOR1>(xr, S2);
    quad_fmac_dpp<DPP_XOR1>(xi, S2);
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = float2{xr[k], xi[k]};
}

// Forward 1024-point FFT of the row held in a[] (see header); T is this
// wave's transpose region.  On return x[k'] = X[b0 + 16 k'],
// b0 = (t >> 2) + 256 c(t & 3).
__device__ __forceinline__ void row_fft(float2 (&a)[16], int t, float2 *T, const float2 *tw,
                                        float2 (&x)[16]) {
    fft_reg<16, false>(a);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) a[k2] = cmul(a[k2], tw[t * TW1P + k2]);
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) T[k2 * TP + t] = a[k2];
    wave_lds_sync();
    const int q = t >> 2, qa = t & 3;
#pragma unroll
    for (int l = 0; l < 16; ++l) x[l] = T[q * TP + qa + 4 * l];
    wave_lds_sync();
    fft_reg<16, false>(x);
    const float2 *tw2 = tw + TW1BUF + qa * TW2P;
    const float g = quad_g(qa);
    x[0] = float2{g * x[0].x, g * x[0].y};
#pragma unroll
    for (int k = 1; k < 16; ++k) x[k] = cmul(x[k], tw2[k]);
    quad_dft(x, qa);
}

__device__ __forceinline__ int lane_bin0(int t) {
    const int qa = t & 3;
    return (t >> 2) + 256 * ((qa >> 1) + 2 * (qa & 1));
}

// Channel estimates of one (frame, antenna row) in "lane order": the 16 bins
// lane t owns (b0(t) + 16 k) as 8 float4 pairs, pair i of lane t at float4
// index i*64 + t -- one contiguous 1 KiB wave load per pair.  Same 8 KiB per
// row as the bin layout; written by k_ls_td1024, read by k_mrc_td1024.
__device__ __forceinline__ void hc_store(float4 *__restrict__ dst, int t, const float2 (&h)[16]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
        dst[i * 64 + t] = float4{h[2 * i].x, h[2 * i].y, h[2 * i + 1].x, h[2 * i + 1].y};
}
__device__ __forceinline__ void hc_load(const float4 *__restrict__ src, int t, float2 (&h)[16]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float4 v = src[i * 64 + t];
        h[2 * i] = float2{v.x, v.y};
        h[2 * i + 1] = float2{v.z, v.w};
    }
}

// ---------------------------------------------------------------------------
// In-launch hand-off of per-frame estimates (the one-launch frame demod
// kernels, k_demod_td*): cdna_hip_programming.md Guideline 16, R1 in its
// write-through form.  The producer stores the payload with sc1 (write-
// through, aux 16 on the buffer / atomic stores -- compiler-generated, so
// the hazard recognizer sees the store-data registers), every storing wave
// drains vmcnt, a workgroup barrier, then ONE lane stores the 64-bit flag
// (relaxed, agent scope).  The consumer polls the flag with one lane
// (relaxed, agent scope, s_sleep between polls, bounded by the 100 MHz wall
// clock), then ONE agent acquire, vmcnt(0) and a workgroup barrier before
// any load of the payload.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
constexpr long long SPIN_TICKS = 200000;  // 2 ms at 100 MHz (A/B build: OFDM_AB_DEMOD_SPIN)

// 16 B {a, b} at byte offset off of [base, base + bytes), write-through
__device__ __forceinline__ void store16_wt(const void *base, int bytes, int off, float2 a, float2 b) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
    const v4i v = {__builtin_bit_cast(int, a.x), __builtin_bit_cast(int, a.y), __builtin_bit_cast(int, b.x),
                   __builtin_bit_cast(int, b.y)};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
}
__device__ __forceinline__ void store8_wt(float2 *p, float2 v) {
    __hip_atomic_store((gu64 *)(p), __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store4_wt(float *p, float v) {
    __hip_atomic_store((gu32 *)(p), __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// producer, every thread of the workgroup: its stores drained, barrier, one
// lane publishes
__device__ __forceinline__ void publish_flag(unsigned long long *flag, unsigned long long epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store((gu64 *)(flag), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ bool wait_flag(unsigned long long *flag, unsigned long long epoch, long long ticks) {
    const long long t0 = wall_clock64();
    while (__hip_atomic_load((gu64 *)(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
        if (wall_clock64() - t0 >= ticks) return false;
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

// consumer, every thread of the workgroup: thread 0 waits for flags f0..fl,
// acquires; returns whether they were seen (false: the bounded wait expired
// -- the caller estimates the frames itself, then calls acquire_all()).
// seen: an LDS word no other code touches before the caller's next barrier.
// seen_before: thread 0 already read every flag at epoch (an early look).
__device__ __forceinline__ bool consume_flags(unsigned long long *flags, long long f0, long long fl,
                                              unsigned long long epoch, long long ticks, int *seen,
                                              bool seen_before = false) {
    if (threadIdx.x == 0) {
        bool ok = true;
        if (!seen_before)
            for (long long f = f0; f <= fl && ok; ++f) ok = wait_flag(flags + f, epoch, ticks);
        *seen = ok ? 1 : 0;
        if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const bool ok = *seen != 0;
    __syncthreads();  // every wave has read the word before it may be reused
    return ok;
}
// after the workgroup wrote an estimate itself: drain, acquire, barrier
__device__ __forceinline__ void acquire_all() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Work tickets: which logical block a workgroup processes is decided at run
// time, not fixed by blockIdx.  Blocks are dealt to the 8 XCDs round-robin
// by the hardware, so with a static map every XCD gets 1/8 of the blocks and
// the kernel ends when the SLOWEST XCD does (round-5 stamps, csrc/diag.hpp:
// per-XCD workgroup lifetimes up to 10 % apart at the headline shape and at
// C = 4096, at equal clocks -- a memory-side difference).  The blocks are
// cut into 8 contiguous ranges, one per XCD (a frame's consecutive blocks
// keep sharing one L2).  The first k0 blocks of range y go statically to
// the workgroups with (index & 7) == y, (index >> 3) < k0 -- the first round
// (k_demod_td1024: the first two), which would otherwise queue on the
// counters all at once; every later block
// is a ticket: a workgroup takes the next one of its own XCD's range (the
// XCC_ID register; speed only) and, once that range is exhausted, of the
// other ranges in turn (one atomic add per block taken).  The grid is
// over-subscribed (ticket_grid: + 25 % + 64 workgroups); a workgroup that
// finds every range exhausted exits at once.  Every block is processed
// exactly once whatever the placement or dispatch order.
// Counters: one set of 8 words (one 128-B line each) in the workspace's
// ticket area, written by nothing but ticketed launches -- but the memory is
// the caller's, and a word may hold anything when a launch starts (an earlier
// launch's count, an estimate of another geometry written over it, a freed
// and re-used allocation).  So a count is tagged: word = tag << 32 | count,
// tag = a per-launch value (never 0; Tickets, launch.hpp).  The first
// workgroup of a launch to meet a range's word with another tag claims it
// with ONE compare-and-swap to (tag, 1) and takes ticket 0; every later one
// adds 1 (the counts stay below 2^32: units + grid < 2^31).  No host
// registry, no zeroing launch, no parity: a stale or garbage word is never
// consumed as a count.  Two launches counting in one word at once (two
// streams sharing a workspace, against the header's contract) show up as a
// foreign tag in a fetch_add result: that launch raises TK_FOREIGN in the
// host-mapped status word (the host returns OFDM_E_DEVICE at the next call)
// and takes nothing more from that range.
// ---------------------------------------------------------------------------
constexpr int TICKET_STRIDE = 16;            // u64 words between counters (128 B)
constexpr int HWREG_XCC_ID = (31 << 11) | 20;
__device__ __forceinline__ long long ticket_range_count(long long nb, long long per, unsigned y) {
    const long long lo = (long long)y * per;
    return nb - lo < per ? (nb - lo > 0 ? nb - lo : 0) : per;
}
__device__ __forceinline__ void ticket_fault(const Tickets &tk, unsigned why) {
    if (tk.status) __hip_atomic_store((gu32 *)tk.status, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// ticket t of range y (t in [0, units)), or -1: none left in the range, -2:
// give up on the range (a fault was raised)
__device__ __forceinline__ long long take_ticket(const Tickets &tk, unsigned y, long long units) {
    gu64 *p = (gu64 *)(tk.set + y * TICKET_STRIDE);
    const unsigned long long mine = (unsigned long long)tk.tag << 32;
    unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int tries = 0; (v >> 32) != tk.tag; ++tries) {  // not counted in by this launch yet: claim it
        if (tries == 64) {
            ticket_fault(tk, TK_CONTENDED);
            return -2;
        }
        if (__hip_atomic_compare_exchange_strong(p, &v, mine | 1ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return 0;
    }
    if ((long long)(unsigned)v >= units) return -1;
    const unsigned long long r = __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((r >> 32) != tk.tag) {
        ticket_fault(tk, TK_FOREIGN);
        return -2;
    }
    const long long t = (long long)(unsigned)r;
    if (t < units) return t;
    if (t > units + (long long)gridDim.x) ticket_fault(tk, TK_RANGE);
    return -1;
}
// thread 0 of workgroup index pb (0-based among the ticketed workgroups):
// the unit (b << 2) | m of block b -- m = 0 the whole block; with split > 0
// the last `split` blocks of every range are dealt as two half units each,
// m = 1 and 2 (their first and second halves of symbols), so that the
// schedule ends on units half as long (k_demod_td1024); -1: none left.
// Every block index formed is in [0, nb).
__device__ __forceinline__ long long take_unit(const Tickets &tk, long long nb, long long k0, long long pb,
                                               long long split) {
    const long long per = (nb + 7) / 8;
    if (pb < 8 * k0) {  // the static first round(s)
        const unsigned y = (unsigned)(pb & 7);
        const long long k = pb >> 3, cnt = ticket_range_count(nb, per, y);
        if (k < (cnt < k0 ? cnt : k0)) return ((long long)y * per + k) << 2;
    }
    const unsigned x = (unsigned)__builtin_amdgcn_s_getreg(HWREG_XCC_ID) & 7u;
    for (int j = 0; j < 8; ++j) {
        const unsigned y = (x + (unsigned)j) & 7u;
        const long long cnt = ticket_range_count(nb, per, y), s0 = cnt < k0 ? cnt : k0;
        const long long avail = cnt - s0;  // ticketed blocks of range y
        if (avail <= 0) continue;
        const long long ns = split < avail ? split : avail, whole = avail - ns;
        const long long t = take_ticket(tk, y, whole + 2 * ns);
        if (t < 0) continue;
        const long long b0 = (long long)y * per + s0;
        if (t < whole) return (b0 + t) << 2;
        const long long u = t - whole;
        return ((b0 + whole + (u >> 1)) << 2) | (1 + (u & 1));
    }
    return -1;
}
// the workgroup's unit: thread 0 takes it, everyone reads it from `slot` (an
// LDS word nothing else touches before the caller's next barrier);
// SGPR-uniform result.  Workgroup 0 (a static block of the first round,
// which takes no ticket) claims the 8 counters for this launch -- (tag, 0)
// -- about a block's time before the first ticket is taken, so that the
// tickets normally meet their tag and cost one add, as untagged counters did
// (the compare-and-swap claim costs 1.3 % at configs[1] without it, profiles/
// r6/r6a_split_estimator_ab_cfg1.jsonl "tk").  Should the claim land after
// tickets were taken, it re-deals them: blocks processed twice, the same
// bytes stored twice; no unit is ever skipped.
__device__ __forceinline__ long long wg_take_unit(const Tickets &tk, long long nb, long long k0, long long pb,
                                                  long long split, long long *slot) {
    if (threadIdx.x == 0) {
        if (pb == 0) {
#pragma unroll
            for (int y = 0; y < 8; ++y)
                __hip_atomic_store((gu64 *)(tk.set + y * TICKET_STRIDE), (unsigned long long)tk.tag << 32,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *slot = take_unit(tk, nb, k0, pb, split);
    }
    __syncthreads();
    const long long v = *slot;
    const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xffffffffll));
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// whole blocks only: the block index, -1 when none is left
__device__ __forceinline__ long long wg_take_block(const Tickets &tk, long long nb, long long k0, long long pb,
                                                   long long *slot) {
    const long long u = wg_take_unit(tk, nb, k0, pb, 0, slot);
    return u < 0 ? u : u >> 2;
}
// The over-subscribed grid of a ticketed kernel: every workgroup takes at
// most one unit and exits only once every range is exhausted, so a grid of
// at least as many workgroups as units (nb blocks + one extra per split
// block: split_units = 8 x split at most) processes every unit whatever the
// placement; + 25 % + 64 so that fast XCDs find workgroups to take more.
inline long long ticket_grid(long long nb, long long split_units = 0) { return nb + split_units + nb / 4 + 64; }
// static blocks per XCD range: the resident workgroups of one XCD (per_cu
// workgroups on each of its CUs), i.e. the first round
inline long long ticket_k0(int per_cu) {
    static const int cus = [] {
        int dev = 0, n = 256;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n = 256;
        return n;
    }();
    return (long long)per_cu * cus / 8;
}

// Twiddle tables and the two FFT halves in the LDS layout of the HLDS
// kernels (k_mrc_td1024_hlds, frame_td2048.hip); see frame_td.hip.
namespace hlds {
constexpr int TW1S = 15 * 64;
constexpr int TW2S = 16 * 4;
constexpr int TP = 68;
constexpr int TS = 16 * TP;
constexpr int WAVES = 8;
constexpr size_t LDS_BYTES = (TW1S + TW2S + WAVES * TS) * sizeof(float2) + 256 * sizeof(float4);
static_assert(LDS_BYTES == 81920, "two workgroups per CU");

// slot of Hc float4 j (0..511) of the staged row; T0 = first transpose image
__device__ __forceinline__ float4 *hslot(float2 *T0, float4 *hfree, int j) {
    if (j < 256) return hfree + j;
    const int jj = j - 256;  // wave image jj>>5, row (jj>>1)&15, tail half jj&1
    return reinterpret_cast<float4 *>(T0 + (jj >> 5) * TS + ((jj >> 1) & 15) * TP + 64 + 2 * (jj & 1));
}

__device__ __forceinline__ void fill(float2 *tw1, float2 *tw2) {
    for (int i = threadIdx.x; i < TW1S; i += blockDim.x) {
        const int k2 = 1 + i / 64, t = i % 64;
        tw1[i] = g_tw[((t * k2) & (C - 1)) * (OFDM_TW_N / C)];
    }
    for (int i = threadIdx.x; i < TW2S; i += blockDim.x) {
        const int k = i / 4, a = i % 4;
        const float2 w = g_tw[((16 * a * k) & (C - 1)) * (OFDM_TW_N / C)];
        const float g = quad_g(a);
        tw2[i] = float2{g * w.x, g * w.y};
    }
}
// fill() in two halves for 512-thread workgroups: fill_load issues this
// thread's (at most 3) table loads, fill_store writes the same values fill()
// does -- the loads' latency overlaps whatever the caller puts between (the
// receivers' work ticket).
struct FillRegs {
    float2 v[3];
};
__device__ __forceinline__ void fill_load(FillRegs &f) {
    const int i0 = threadIdx.x, i1 = threadIdx.x + 512;
    auto w1 = [](int i) { return g_tw[(((i % 64) * (1 + i / 64)) & (C - 1)) * (OFDM_TW_N / C)]; };
    f.v[0] = w1(i0);
    f.v[1] = i1 < TW1S ? w1(i1) : float2{0.f, 0.f};
    f.v[2] = i0 < TW2S ? g_tw[((16 * (i0 % 4) * (i0 / 4)) & (C - 1)) * (OFDM_TW_N / C)] : float2{0.f, 0.f};
}
__device__ __forceinline__ void fill_store(float2 *tw1, float2 *tw2, const FillRegs &f) {
    const int i0 = threadIdx.x, i1 = threadIdx.x + 512;
    tw1[i0] = f.v[0];
    if (i1 < TW1S) tw1[i1] = f.v[1];
    if (i0 < TW2S) {
        const float g = quad_g(i0 % 4);
        tw2[i0] = float2{g * f.v[2].x, g * f.v[2].y};
    }
}
static_assert(TW1S <= 1024 && TW2S <= 512, "fill_load covers the tables with 512 threads");
// index of (row, col) in a transpose image
__device__ __forceinline__ int swz(int row, int col) { return row * TP + col; }

// Twiddles w^k, k = 1..15, of a per-lane base w (one LDS read) by two
// interleaved recurrences of depth 7 (w^(k+2) = w^k w^2) instead of 15 table
// reads: register-starved kernels otherwise issue the reads one round trip
// at a time.  v[k] *= s w^k for k >= 1.
template <int N>
__device__ __forceinline__ void tw_powers(pk::v2f (&v)[N], pk::v2f w, pk::v2f sw) {
    const pk::v2f w2 = pk::cmul(w, w);
    pk::v2f po = sw, pe = pk::cmul(sw, w);
    v[1] = pk::cmul(v[1], po);
    v[2] = pk::cmul(v[2], pe);
#pragma unroll
    for (int k = 3; k < N; k += 2) {
        po = pk::cmul(po, w2);
        v[k] = pk::cmul(v[k], po);
        if (k + 1 < N) {
            pe = pk::cmul(pe, w2);
            v[k + 1] = pk::cmul(v[k + 1], pe);
        }
    }
}

// first half: radix-16 over m, twiddles, transpose write.  PK: packed-f32
// butterflies and twiddle multiplies (pk.hpp).  TWR: twiddles by recurrence
// from W1024^t (tw_powers) instead of 15 table reads.
template <int PK = 0, bool TWR = false>
__device__ __forceinline__ void row_fft_a(float2 (&a)[16], int t, float2 *T, const float2 *tw1) {
    if constexpr (TWR) {
        pk::v2f v[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = pk::V(a[m]);
        if constexpr ((PK & 1) != 0) {
            pk::fft_reg<16>(v);
        } else {
#pragma unroll
            for (int m = 0; m < 16; ++m) a[m] = pk::F(v[m]);
            fft_reg<16, false>(a);
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = pk::V(a[m]);
        }
        const pk::v2f w = pk::V(tw1[t]);  // W1024^t
        tw_powers(v, w, w);
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) T[swz(k2, t)] = pk::F(v[k2]);
        return;
    }
    if constexpr (PK & 1) {
        pk::v2f v[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = pk::V(a[m]);
        pk::fft_reg<16>(v);
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) v[k2] = pk::cmul(v[k2], pk::V(tw1[(k2 - 1) * 64 + t]));
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) T[swz(k2, t)] = pk::F(v[k2]);
        return;
    }
    fft_reg<16, false>(a);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) a[k2] = cmul(a[k2], tw1[(k2 - 1) * 64 + t]);
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) T[swz(k2, t)] = a[k2];
}
// second half: transpose read, radix-16, twiddles, quad DFT.  TWR: the
// twiddles g(a) W64^(a k) by recurrence from tw2[4 + a] = g(a) W64^a.
template <int PK = 0, bool TWR = false>
__device__ __forceinline__ void row_fft_b(int t, float2 *T, const float2 *tw2, float2 (&x)[16]) {
    wave_lds_sync();
    const int q = t >> 2, qa = t & 3;
#pragma unroll
    for (int l = 0; l < 16; ++l) x[l] = T[swz(q, qa + 4 * l)];
    wave_lds_sync();
    const float g = quad_g(qa);
    if constexpr (TWR) {
        pk::v2f v[16];
        if constexpr ((PK & 2) != 0) {
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = pk::V(x[m]);
            pk::fft_reg<16>(v);
        } else {
            fft_reg<16, false>(x);
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = pk::V(x[m]);
        }
        v[0] = pk::scale(v[0], g);
        const pk::v2f gw = pk::V(tw2[4 + qa]);  // g W64^a
        tw_powers(v, pk::scale(gw, g), gw);
#pragma unroll
        for (int m = 0; m < 16; ++m) x[m] = pk::F(v[m]);
    } else if constexpr (PK & 2) {
        pk::v2f v[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = pk::V(x[m]);
        pk::fft_reg<16>(v);
        v[0] = pk::scale(v[0], g);
#pragma unroll
        for (int k = 1; k < 16; ++k) v[k] = pk::cmul(v[k], pk::V(tw2[k * 4 + qa]));
#pragma unroll
        for (int m = 0; m < 16; ++m) x[m] = pk::F(v[m]);
    } else {
        fft_reg<16, false>(x);
        x[0] = float2{g * x[0].x, g * x[0].y};
#pragma unroll
        for (int k = 1; k < 16; ++k) x[k] = cmul(x[k], tw2[k * 4 + qa]);
    }
    quad_dft(x, qa);
}
// Transpose images for 16-B reads (the C = 2048 / 4096 receivers, whose LDS
// budget has room for the wider pitch): 16 rows of pitch TP16 = 72 float2, row
// element c = a + 4 l (a < 4) at position 8 (l >> 1) + 2 a + (l & 1), so
// that the second FFT half reads lane (q, a)'s values l = 2 j, 2 j + 1 as
// ONE 16-B ds_read_b128 at q TP16 + 8 j + 2 a (4 LDS cycles; the hlds image
// of pitch 68 gives ds_read2_b64, 8 cycles: MI355X_MICROARCH.md LDS table).
// Conflict-free both ways: a transpose-write row covers 16 lanes x 8 B
// contiguously per lane group, and the four rows a ds_read_b128 lane group
// reads start 16 dwords apart mod 64 (pitch 144 dwords).
constexpr int TP16 = 72;
constexpr int TS16 = 16 * TP16;
__device__ __forceinline__ int perm16(int c) { return 8 * (c >> 3) + 2 * (c & 3) + ((c >> 2) & 1); }
__device__ __forceinline__ void fa_write16(const pk::v2f (&v)[16], int pt, float2 *T) {
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) T[k2 * TP16 + pt] = pk::F(v[k2]);
}
__device__ __forceinline__ void fb_read16(int t, const float2 *T, pk::v2f (&v)[16]) {
    const float4 *s = reinterpret_cast<const float4 *>(T + (t >> 2) * TP16 + 2 * (t & 3));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float4 x = s[4 * j];  // float2 offset 8 j
        v[2 * j] = pk::V(float2{x.x, x.y});
        v[2 * j + 1] = pk::V(float2{x.z, x.w});
    }
}

// The two FFT1024 stages of hlds::row_fft_a / row_fft_b (PK = 3, TW = 3:
// packed butterflies, twiddles by recurrence) split at the transpose, so that
// the IL variants of the C = 2048 / 4096 rows can put one transform's compute between the other's
// LDS write and read (A/B build only).
// w1 = W1024^t (tw1[t]) and gw = g(a) W64^a (tw2[4 + a]) are per-lane row
// invariants, read from LDS once per kernel: an LDS read inside the pipeline
// would make every later wait on it a wait for the whole transpose in flight.
// Twiddles s W^k, k = 1..15, from exact table anchors A_k = s W^k for
// k = 1, 4, 8, 12 and the base W: every other power is one anchor times W,
// W^2 or W^3 (recursion depth <= 3 instead of tw_powers' 7, so the error
// stays within a few ulp -- tw_powers' up to 8e-7 pushed single-antenna
// (R = 1) outputs past the 1e-5 element-wise parity bound).
struct TwAnchors {
    pk::v2f w, a1, a4, a8, a12;
};
__device__ __forceinline__ void tw_anchored(pk::v2f (&v)[16], const TwAnchors &c) {
    const pk::v2f w2 = pk::cmul(c.w, c.w), w3 = pk::cmul(w2, c.w);
    v[1] = pk::cmul(v[1], c.a1);
    v[2] = pk::cmul(v[2], pk::cmul(c.a1, c.w));
    v[3] = pk::cmul(v[3], pk::cmul(c.a1, w2));
#pragma unroll
    for (int j = 1; j < 4; ++j) {
        const pk::v2f a = j == 1 ? c.a4 : j == 2 ? c.a8 : c.a12;
        v[4 * j] = pk::cmul(v[4 * j], a);
        v[4 * j + 1] = pk::cmul(v[4 * j + 1], pk::cmul(a, c.w));
        v[4 * j + 2] = pk::cmul(v[4 * j + 2], pk::cmul(a, w2));
        v[4 * j + 3] = pk::cmul(v[4 * j + 3], pk::cmul(a, w3));
    }
}
// The anchors of the two FFT1024 stages for lane t, from the hlds tables:
// stage A: W1024^(t k) = tw1[(k - 1) * 64 + t]; stage B: g(a) W64^(a k) =
// tw2[k * 4 + a] (g = +-1, so W = g * tw2[4 + a] is exact).
__device__ __forceinline__ TwAnchors anchors_a(const float2 *tw1, int t) {
    const pk::v2f w = pk::V(tw1[t]);
    return TwAnchors{w, w, pk::V(tw1[3 * 64 + t]), pk::V(tw1[7 * 64 + t]), pk::V(tw1[11 * 64 + t])};
}
__device__ __forceinline__ TwAnchors anchors_b(const float2 *tw2, int t) {
    const int qa = t & 3;
    const pk::v2f gw = pk::V(tw2[4 + qa]);
    return TwAnchors{pk::scale(gw, quad_g(qa)), gw, pk::V(tw2[16 + qa]), pk::V(tw2[32 + qa]), pk::V(tw2[48 + qa])};
}

__device__ __forceinline__ void fa_compute(pk::v2f (&v)[16], pk::v2f w1) {
    pk::fft_reg<16>(v);
    tw_powers(v, w1, w1);
}
__device__ __forceinline__ void fa_compute(pk::v2f (&v)[16], const TwAnchors &c) {
    pk::fft_reg<16>(v);
    tw_anchored(v, c);
}
__device__ __forceinline__ void fa_write(const pk::v2f (&v)[16], int t, float2 *T) {
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) T[swz(k2, t)] = pk::F(v[k2]);
}
__device__ __forceinline__ void fb_read(int t, const float2 *T, pk::v2f (&v)[16]) {
    const int q = t >> 2, qa = t & 3;
#pragma unroll
    for (int l = 0; l < 16; ++l) v[l] = pk::V(T[swz(q, qa + 4 * l)]);
}
__device__ __forceinline__ void fb_compute(pk::v2f (&v)[16], pk::v2f gw, int t, float2 (&x)[16]) {
    const int qa = t & 3;
    const float g = quad_g(qa);
    pk::fft_reg<16>(v);
    v[0] = pk::scale(v[0], g);
    tw_powers(v, pk::scale(gw, g), gw);
#pragma unroll
    for (int m = 0; m < 16; ++m) x[m] = pk::F(v[m]);
    quad_dft(x, qa);
}
__device__ __forceinline__ void fb_compute(pk::v2f (&v)[16], const TwAnchors &c, int t, float2 (&x)[16]) {
    const int qa = t & 3;
    pk::fft_reg<16>(v);
    v[0] = pk::scale(v[0], quad_g(qa));
    tw_anchored(v, c);
#pragma unroll
    for (int m = 0; m < 16; ++m) x[m] = pk::F(v[m]);
    quad_dft(x, qa);
}

}  // namespace hlds

}  // namespace td1024
}  // namespace ofdm
