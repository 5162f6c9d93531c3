// rfft1024.hpp -- 1024-point forward FFT on one 64-lane wave with no LDS
// transpose (CDNA4: v_permlane32_swap / v_permlane16_swap + DPP).
//
// Lane t holds x[t + 64 m], m < 16 (the same coalesced row load as
// wave_fft1024.hpp).  Four-step, N = 16 x 64:
//   A[t][k2] = FFT16_m(x[t + 64 m]) * W1024^(t k2)                 registers
//   X[k2 + 16 k1] = DFT64_t(A[t][k2])
// and the DFT64 over the lanes, t = t_lo + 16 t_hi, k1 = k_hi + 4 k_lo:
//   1. the two high lane bits (t_hi) are swapped into the register index
//      (v_permlane32_swap on register pairs j, j^8; v_permlane16_swap on
//      j, j^4), so that register j = (j3 j2 j1 j0) of lane L holds t_hi =
//      (j3 j2) of k2 = j0 + 2 j1 + 4 L4 + 8 L5;
//   2. DFT4 over t_hi in registers (output k_hi in register bits 3..2),
//      times W64^(t_lo k_hi);
//   3. DFT16 over t_lo = lane bits 0..3 (decimation in frequency across the
//      lanes of a 16-lane row): bit 3 by row_ror:8, bit 2 by row_ror:12 /
//      row_ror:4 under complementary bank masks, bits 1..0 by the quad DFT of
//      wave_fft1024.hpp (quad_perm DPP), twiddles as per-lane constants.
// Lane L's register j then holds X[b], b = k2 + 16 (k_hi + 4 k_lo) with
//   k_lo = L3 + 2 L2 + 4 c(L1 L0),  c(a) = (a >> 1) + 2 (a & 1)   (rfft_bin).
#pragma once
#include "pk.hpp"
#include "wave_fft1024.hpp"

namespace ofdm {
namespace rfft {

using pk::v2f;

// bin of register j in lane L
__host__ __device__ __forceinline__ constexpr int rfft_bin(int L, int j) {
    const int k2 = (j & 3) + 4 * ((L >> 4) & 1) + 8 * ((L >> 5) & 1);
    const int khi = j >> 2;
    const int a = L & 3;
    const int klo = ((L >> 3) & 1) + 2 * ((L >> 2) & 1) + 4 * ((a >> 1) + 2 * (a & 1));
    return k2 + 16 * (khi + 4 * klo);
}

// Per-lane constants of the cross-lane stages (computed once per kernel).
struct Consts {
    v2f w1024;       // W1024^t (twiddles by recurrence, fft1024<true>)
    v2f w1, w2, w3;  // W64^(t_lo k_hi), k_hi = 1..3
    v2f c1;          // stage 1 (lane bit 3): 1, or -W16^(t_lo & 7)
    v2f c2;          // stage 2 (lane bit 2): g(a) (W8^(t_lo & 3) if bit 2), g of the quad DFT folded in
    float s1;        // +1 / -1 (lane bit 3)
};

__device__ __forceinline__ Consts make_consts(int t) {
    Consts c;
    const int tl = t & 15;
    c.w1024 = pk::V(g_tw[t * (OFDM_TW_N / 1024)]);
    c.w1 = pk::V(g_tw[(tl * 1) * (OFDM_TW_N / 64)]);
    c.w2 = pk::V(g_tw[(tl * 2) * (OFDM_TW_N / 64)]);
    c.w3 = pk::V(g_tw[(tl * 3) * (OFDM_TW_N / 64)]);
    const bool b3 = (tl >> 3) & 1, b2 = (tl >> 2) & 1;
    const float2 w16 = g_tw[(tl & 7) * (OFDM_TW_N / 16)];
    c.c1 = b3 ? (v2f){-w16.x, -w16.y} : (v2f){1.f, 0.f};
    c.s1 = b3 ? -1.f : 1.f;
    const float2 w8 = g_tw[(tl & 3) * (OFDM_TW_N / 8)];
    const float g = td1024::quad_g(tl & 3);
    c.c2 = b2 ? (v2f){g * w8.x, g * w8.y} : (v2f){g, 0.f};
    return c;
}

template <int CTRL>
__device__ __forceinline__ void swap_pair(float &p, float &q) {
    unsigned a = __builtin_bit_cast(unsigned, p), b = __builtin_bit_cast(unsigned, q);
    auto r = CTRL == 32 ? __builtin_amdgcn_permlane32_swap(a, b, false, false)
                        : __builtin_amdgcn_permlane16_swap(a, b, false, false);
    p = __builtin_bit_cast(float, (unsigned)r[0]);
    q = __builtin_bit_cast(float, (unsigned)r[1]);
}

// v[k] = dpp_ror8(v[k]) * s + v[k] for 16 floats (stage 1, in place: each
// instruction reads its partner before writing)
__device__ __forceinline__ void ror8_fmac(float (&v)[16], float s) {
#define OFDM_R8(i) "v_fmac_f32_dpp %" #i ", %" #i ", %16 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
    asm("s_nop 1\n\t" OFDM_R8(0) OFDM_R8(1) OFDM_R8(2) OFDM_R8(3) OFDM_R8(4) OFDM_R8(5) OFDM_R8(6) OFDM_R8(7)
            OFDM_R8(8) OFDM_R8(9) OFDM_R8(10) OFDM_R8(11) OFDM_R8(12) OFDM_R8(13) OFDM_R8(14) OFDM_R8(15)
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
          "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
        : "v"(s));
#undef OFDM_R8
}

// stage 2 (lane bit 2, partner L ^ 4) on 8 floats: w = v + partner on
// lanes with bit 2 clear (banks 0, 2: partner at L + 4 = row_ror:12), w =
// partner - v on lanes with bit 2 set (banks 1, 3: partner at L - 4 =
// row_ror:4); out of place so that both halves read unmodified values.
__device__ __forceinline__ void xor4_bfly8(const float *v, float *w) {
#define OFDM_X4(i, o)                                                              \
    "v_add_f32_dpp %" #o ", %" #i ", %" #i " row_ror:12 row_mask:0xf bank_mask:0x5\n\t" \
    "v_sub_f32_dpp %" #o ", %" #i ", %" #i " row_ror:4 row_mask:0xf bank_mask:0xa\n\t"
    asm("s_nop 1\n\t" OFDM_X4(8, 0) OFDM_X4(9, 1) OFDM_X4(10, 2) OFDM_X4(11, 3) OFDM_X4(12, 4) OFDM_X4(13, 5)
            OFDM_X4(14, 6) OFDM_X4(15, 7)
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7])
        : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
#undef OFDM_X4
}

// Forward FFT of the row in a[] (a[m] = x[t + 64 m]); on return a[j] = X[rfft_bin(t, j)].
// tw1: the hlds W1024^(t k2) table in LDS ([k2 - 1][t], k2 = 1..15); TWR:
// those twiddles by recurrence from c.w1024 instead (no table; tw1 unused).
template <bool TWR = false>
__device__ __forceinline__ void fft1024(float2 (&a)[16], int t, const float2 *tw1, const Consts &c) {
    v2f v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = pk::V(a[m]);
    pk::fft_reg<16>(v);
    if constexpr (TWR) {
        td1024::hlds::tw_powers(v, c.w1024, c.w1024);
    } else {
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) v[k2] = pk::cmul(v[k2], pk::V(tw1[(k2 - 1) * 64 + t]));
    }
    // 1. t5 -> register bit 3, t4 -> register bit 2
    float re[16], im[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) { re[j] = v[j].x; im[j] = v[j].y; }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        swap_pair<32>(re[j], re[j + 8]);
        swap_pair<32>(im[j], im[j + 8]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (j & 4) continue;
        swap_pair<16>(re[j], re[j + 4]);
        swap_pair<16>(im[j], im[j + 4]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (v2f){re[j], im[j]};
    // 2. DFT4 over t_hi = (j3 j2), then W64^(t_lo k_hi)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const v2f e0 = v[g], e1 = v[4 + g], e2 = v[8 + g], e3 = v[12 + g];
        const v2f s02 = pk::add(e0, e2), d02 = pk::sub(e0, e2), s13 = pk::add(e1, e3), d13 = pk::sub(e1, e3);
        v[g] = pk::add(s02, s13);
        v[8 + g] = pk::cmul(pk::sub(s02, s13), c.w2);
        v[4 + g] = pk::cmul(pk::add_mi(d02, d13), c.w1);
        v[12 + g] = pk::cmul(pk::sub_mi(d02, d13), c.w3);
    }
    // 3. DFT16 over lane bits 0..3
#pragma unroll
    for (int j = 0; j < 16; ++j) { re[j] = v[j].x; im[j] = v[j].y; }
    ror8_fmac(re, c.s1);
    ror8_fmac(im, c.s1);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const v2f x = pk::cmul((v2f){re[j], im[j]}, c.c1);
        re[j] = x.x;
        im[j] = x.y;
    }
    float wr[16], wi[16];
    xor4_bfly8(re, wr);
    xor4_bfly8(re + 8, wr + 8);
    xor4_bfly8(im, wi);
    xor4_bfly8(im + 8, wi + 8);
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = pk::F(pk::cmul((v2f){wr[j], wi[j]}, c.c2));
    td1024::quad_dft(a, t & 3);
}

}  // namespace rfft
}  // namespace ofdm
