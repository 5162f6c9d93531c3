// pk.hpp -- packed-f32 complex arithmetic for CDNA4 (gfx950).
//
// A complex float {re, im} lives in an aligned VGPR pair, which is exactly
// the operand of the VOP3P f32 instructions v_pk_add_f32 / v_pk_mul_f32 /
// v_pk_fma_f32: one instruction does both halves at the full f32 issue rate
// (2 flops/lane/cycle per FMA half -- the packed rate behind MI355X's
// 157 TF vector peak).  op_sel / op_sel_hi pick which half of each source
// feeds the low / high result and neg_lo / neg_hi negate it, so swaps and
// sign flips cost nothing:
//   complex add / sub        1 instruction   (scalar: 2)
//   u +/- (-i) v             1 instruction   (scalar: 2, after a swap)
//   complex multiply         2 instructions  (scalar: 4)
//   acc += x * h             2 instructions  (scalar: 4)
// The compiler's own vectoriser gets the swaps and constants wrong (extra
// v_mov / v_xor / constant multiplies), hence inline asm for the shuffled
// forms.  No DPP or transcendental op is emitted here, so none of the
// VALU -> DPP / trans hazards apply between these instructions.
#pragma once
#include "common.hpp"

namespace ofdm {
namespace pk {

typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2f V(float2 a) { return __builtin_bit_cast(v2f, a); }
__device__ __forceinline__ float2 F(v2f a) { return __builtin_bit_cast(float2, a); }

__device__ __forceinline__ v2f add(v2f a, v2f b) { return a + b; }
__device__ __forceinline__ v2f sub(v2f a, v2f b) { return a - b; }

// u + (-i) v = (u.x + v.y, u.y - v.x)
__device__ __forceinline__ v2f add_mi(v2f u, v2f v) {
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]"
        : "=v"(r) : "v"(u), "v"(v));
    return r;
}
// u - (-i) v = (u.x - v.y, u.y + v.x)
__device__ __forceinline__ v2f sub_mi(v2f u, v2f v) {
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
        : "=v"(r) : "v"(u), "v"(v));
    return r;
}

// Each multi-instruction form is ONE asm statement: hipcc pads one wait
// state (s_nop 0, a 4-cycle issue slot) after an ;;#ASMEND whose outputs the
// next instruction reads, so two statements chained through a temporary cost
// a nop each time; VALU -> VALU needs no wait state inside the string.
// a * b: r = (a.x b.x, a.x b.y); r += (a.y (-b.y), a.y b.x) -- the product
// accumulated in the (early-clobber) result register itself, no temporary
// (a temporary freed at ;;#ASMEND and reused by the next statement draws a
// pad as well)
__device__ __forceinline__ v2f cmul(v2f a, v2f b) {
    v2f r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=&v"(r) : "v"(a), "v"(b));
    return r;
}
// a * w with a wave-uniform (compile-time) w held in an SGPR pair
__device__ __forceinline__ v2f cmul_s(v2f a, v2f w) {
    v2f r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=&v"(r) : "v"(a), "s"(w));
    return r;
}
// cmul_s that the compiler may not hoist out of a loop (a loop-invariant
// twiddle set kept live across the loop costs two VGPRs per twiddle)
__device__ __forceinline__ v2f cmul_s_v(v2f a, v2f w) {
    v2f r;
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
                 "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
                 : "=&v"(r) : "v"(a), "s"(w));
    return r;
}
// acc += x * h.  Two instructions in one statement: the second reads x and h
// after the first has written acc, so acc is early-clobber ("+&v") and can
// never share a register with x or h (e.g. mac(a, a, h)).
__device__ __forceinline__ void mac(v2f &acc, v2f x, v2f h) {
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "+&v"(acc) : "v"(x), "v"(h));
}
// v * (a * b): the twiddle a * b formed and applied in one statement
// (twiddle generation chains: no pad between the product and its use)
#define OFDM_PK_CMUL2(DST, A, B)                                                          \
    "v_pk_mul_f32 " DST ", " A ", " B " op_sel_hi:[0,1]\n\t"                              \
    "v_pk_fma_f32 " DST ", " A ", " B ", " DST " op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
__device__ __forceinline__ v2f cmul3(v2f v, v2f a, v2f b) {
    v2f ab, r;
    asm(OFDM_PK_CMUL2("%1", "%2", "%3") OFDM_PK_CMUL2("%0", "%4", "%1")
        : "=&v"(r), "=&v"(ab) : "v"(a), "v"(b), "v"(v));
    return r;
}
// v * (a * w), w wave-uniform (SGPR pair); volatile as cmul_s_v
__device__ __forceinline__ v2f cmul3_s_v(v2f v, v2f a, v2f w) {
    v2f ab, r;
    asm volatile(OFDM_PK_CMUL2("%1", "%2", "%3") OFDM_PK_CMUL2("%0", "%4", "%1")
                 : "=&v"(r), "=&v"(ab) : "v"(a), "s"(w), "v"(v));
    return r;
}
// radix-2 butterfly with a wave-uniform twiddle: (u + v w, u - v w)
__device__ __forceinline__ void bfly_s(v2f &u, v2f &v, v2f w) {
    v2f tv;
    asm(OFDM_PK_CMUL2("%2", "%1", "%3")
        "v_pk_add_f32 %1, %0, %2 neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %0, %0, %2"
        : "+v"(u), "+v"(v), "=&v"(tv) : "s"(w));
}
#undef OFDM_PK_CMUL2
// (x, y) * s for a real s
__device__ __forceinline__ v2f scale(v2f a, float s) { return a * (v2f){s, s}; }

// In-register radix-2 forward FFT of N points per lane (natural order in and
// out), as fft_reg<N, false> (common.hpp) with packed butterflies: twiddle 1
// and -i butterflies are 2 instructions, others 4.
template <int N>
__device__ __forceinline__ void fft_reg(v2f (&a)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int j = bitrev<N>(i);
        if (i < j) { v2f t = a[i]; a[i] = a[j]; a[j] = t; }
    }
#pragma unroll
    for (int len = 2; len <= N; len <<= 1) {
        const int half = len >> 1;
#pragma unroll
        for (int i = 0; i < N; i += len) {
#pragma unroll
            for (int k = 0; k < half; ++k) {
                const v2f u = a[i + k], v = a[i + k + half];
                if (k == 0) {
                    a[i + k] = add(u, v);
                    a[i + k + half] = sub(u, v);
                } else if (4 * k == len) {
                    a[i + k] = add_mi(u, v);
                    a[i + k + half] = sub_mi(u, v);
                } else {
                    const int idx = k * (OFDM_TW_N / len);
                    const v2f w = {kTw.v[2 * idx], kTw.v[2 * idx + 1]};
                    v2f uu = u, vv = v;
                    bfly_s(uu, vv, w);
                    a[i + k] = uu;
                    a[i + k + half] = vv;
                }
            }
        }
    }
}

}  // namespace pk
}  // namespace ofdm
