// fft_any.hip -- FFT lengths beyond the fused receivers: a batched row FFT of
// ANY length C in [2, 8192] (k_fft_any) and the fused any-C MRC (k_mrc_any:
// FFT + combine + normalise + rotate in one HBM pass), for the sizes the
// power-of-two kernels (k_fft_rows, the fused C = 1024 / 2048 / 4096
// receivers) do not cover: 1536 (LTE 15 MHz), 3072, 6144, 600, 1200, odd and
// prime lengths, 8192 and the small powers of two.  The reference transforms
// whatever `dimension` it is built with (ShMemSymBuff.hpp:47) through FFTW
// (fftOneRow, cpuLS.hpp:165-174) or cuFFT (gpuLS.cu:94-97, 377-381), both
// size-generic.  Unnormalised, forward sign -1 (inverse +1, then `scale`).
//
// Algorithm (C = p_1 p_2 ... p_n, one Stockham stage per factor):
//   after the stages with radices whose product is L', the row holds
//   y[m][k] = DFT_{L'} of the subsequence x[m + n M'] (M' = C / L'), stored
//   at m L' + k.  A stage of radix p (L = L' p, cp = C / p) forms, for each
//   butterfly b = m L' + k1 (b < cp):
//     a_t = W_L^{t k1} y[b + t cp],  t < p
//     y'[m L + k1 + L' k2] = sum_t W_p^{t k2} a_t,  k2 < p
//   which ends in natural order (L = C).  Radices 8, 4, 2 run as in-register
//   FFTs with compile-time twiddles (common.hpp fft_reg), 3, 5, 7 as direct
//   DFTs with their p - 1 roots in registers; any other prime factor runs one
//   output per thread, sum_t W_L^{(t k) mod L} y[b + t cp] over the p inputs,
//   accumulated in double (products of two floats are exact in double).
//
// Layout: a workgroup owns G = CAP / C rows at a time in LDS, two buffers of
// CAP complex (out-of-place stages, one barrier per stage, no values held
// across a barrier, so the stages need few registers and the next row
// group's loads can sit in registers meanwhile).  Twiddles W_C^e = lo[e mod
// 64] * hi[e / 64], both tables (64 + C/64 entries) computed per workgroup in
// double precision and rounded: one complex multiply per twiddle, within an
// ulp of a full table, with no table-sized LDS.  Variants by C: CAP 2048 (256
// threads, 32 KiB, 4 workgroups per CU), 4096 (256 threads, 64 KiB, 2 per
// CU), 8192 (512 threads, 128 KiB, 1 per CU); each thread holds CAP / NT
// elements of a prefetched row group.
#include "common.hpp"
#include "launch.hpp"
#include "pk.hpp"

namespace ofdm {
namespace fany {

// threadIdx.x through a volatile copy: index math derived from it is formed
// where it is used, not hoisted out of the symbol loop (where it was spilled)
__device__ __forceinline__ unsigned tid_here() {
    unsigned r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"((unsigned)threadIdx.x));
    return r;
}

constexpr int MAX_STAGES = 16;
constexpr int TLO = 64;          // low twiddle table: W_C^j, j < 64
constexpr int THI = 8192 / TLO;  // high table: W_C^{64 k}, k < C / 64

// n / d for n < 2^24 as (umulhi(n, m) + n) >> l (round-up magic numbers,
// computed on the host: the stages divide by runtime sizes per butterfly)
struct FDiv {
    unsigned m, l;
};
__device__ __forceinline__ unsigned fdiv(unsigned n, FDiv f) { return (__umulhi(n, f.m) + n) >> f.l; }
inline FDiv make_fdiv(unsigned d) {
    const unsigned l = d > 1 ? 32 - __builtin_clz(d - 1) : 0;
    return FDiv{(unsigned)((((1ull << 32) * ((1ull << l) - d)) / d) + 1), l};
}

struct Stage {
    int p;
    FDiv cp, Lp, L;  // divisors of the stage: C / p, the product of the earlier radices, Lp * p
};
// flat arrays (read by a runtime stage index straight from the kernel
// arguments; an array of structs would be copied to scratch)
struct Plan {
    int C, G, ns;
    FDiv dC;
    int p[MAX_STAGES];
    unsigned m[3][MAX_STAGES], l[3][MAX_STAGES];
};

// LDS capacity (complex elements per buffer) of the variant that takes C,
// its threads per workgroup and the waves per SIMD it is built for
constexpr int cap_of(int C) { return C <= 2048 ? 2048 : C <= 4096 ? 4096 : 8192; }
constexpr int nt_of(int cap) { return cap <= 4096 ? 256 : 512; }
constexpr int wpe_of(int cap) { return cap <= 2048 ? 4 : 2; }
// the fused MRC holds three prefetch / accumulator arrays beside the stages
constexpr int wpe_mrc(int cap) { return cap <= 2048 ? 3 : 2; }

struct Tw {
    const float2 *lo, *hi;
};

// Workgroup barrier that orders LDS only.  __syncthreads() also drains every
// outstanding global load (s_waitcnt vmcnt(0)), which would wait for the next
// row group's prefetch at the first stage barrier: the prefetch would never
// overlap the stages (measured: ~1 TB/s with it, all rows waiting on HBM).
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool INV>
__device__ __forceinline__ float2 twv(const Tw &T, unsigned e) {
    const float2 w = cmul(T.lo[e & (TLO - 1)], T.hi[e / TLO]);
    return INV ? float2{w.x, -w.y} : w;
}

template <int NT>
__device__ __forceinline__ void fill_tables(float2 *lo, float2 *hi, unsigned C) {
    const unsigned nhi = (C + TLO - 1) / TLO;
    for (unsigned i = threadIdx.x; i < TLO + nhi; i += NT) {
        const unsigned e = i < TLO ? i : (i - TLO) * TLO;
        double s, c;
        sincospi(-2.0 * (double)(e % C) / (double)C, &s, &c);
        (i < TLO ? lo[i] : hi[i - TLO]) = float2{(float)c, (float)s};
    }
}

// radices 2, 4, 8: in-register FFT (compile-time twiddles);
// 3, 5, 7: direct DFT with the roots r[j] = W_p^j in registers
// (packed f32: pk.hpp; the inverse 2/4/8-point FFT as conj(FFT(conj(a))))
template <int P, bool INV>
__device__ __forceinline__ void dft_small(float2 (&a)[P], const float2 (&r)[P]) {
    pk::v2f v[P];
#pragma unroll
    for (int t = 0; t < P; ++t) v[t] = pk::V(INV && (P == 2 || P == 4 || P == 8) ? float2{a[t].x, -a[t].y} : a[t]);
    if constexpr (P == 2 || P == 4 || P == 8) {
        pk::fft_reg<P>(v);
#pragma unroll
        for (int t = 0; t < P; ++t) a[t] = INV ? float2{v[t].x, -v[t].y} : pk::F(v[t]);
    } else {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            pk::v2f s = v[0];
#pragma unroll
            for (int t = 1; t < P; ++t) pk::mac(s, v[t], pk::V(r[(t * k) % P]));
            a[k] = pk::F(s);
        }
    }
}

// a[t] *= W_C^{t e}, t = 1..P-1, each twiddle from the two-level table
// (one rounding beyond the table's; powers by products of depth 3 instead
// put single-antenna outputs at C = 6144 past the 1e-5 element-wise bound)
template <int P, bool INV>
__device__ __forceinline__ void twiddle_powers(float2 (&a)[P], const Tw &T, unsigned e) {
#pragma unroll
    for (int t = 1; t < P; ++t) a[t] = pk::F(pk::cmul(pk::V(a[t]), pk::V(twv<INV>(T, t * e))));
}

// one radix-P stage over G rows, src -> dst (caller synchronises after)
template <int P, int NT, bool INV>
__device__ __forceinline__ void stage_small(const float2 *src, float2 *dst, const Tw &T, unsigned C, unsigned G,
                                            unsigned Lp, const Stage &st) {
    const unsigned cp = C / P, nb = G * cp, M = cp / Lp;
    float2 r[P];
#pragma unroll
    for (int j = 0; j < P; ++j) r[j] = (P == 3 || P == 5 || P == 7) ? twv<INV>(T, j * cp) : float2{1.f, 0.f};
    for (unsigned bb = tid_here(); bb < nb; bb += NT) {
        const unsigned g = fdiv(bb, st.cp), b = bb - g * cp, m = fdiv(b, st.Lp), k1 = b - m * Lp;
        const unsigned s0 = g * C + b;
        float2 a[P];
#pragma unroll
        for (int t = 0; t < P; ++t) a[t] = src[s0 + t * cp];
        if (k1 != 0) twiddle_powers<P, INV>(a, T, k1 * M);
        dft_small<P, INV>(a, r);
        const unsigned d0 = g * C + m * Lp * P + k1;
#pragma unroll
        for (int k2 = 0; k2 < P; ++k2) dst[d0 + k2 * Lp] = a[k2];
    }
}

// one stage of any radix p, one output per iteration, double accumulation
template <int NT, bool INV>
__device__ __forceinline__ void stage_any(const float2 *src, float2 *dst, const Tw &T, unsigned C, unsigned G,
                                          unsigned Lp, unsigned p, const Stage &st, FDiv dC) {
    const unsigned L = Lp * p, cp = C / p, M = C / L, n = G * C;
    for (unsigned o = tid_here(); o < n; o += NT) {
        const unsigned g = fdiv(o, dC), pos = o - g * C, m = fdiv(pos, st.L), k = pos - m * L;
        const unsigned k1 = k - fdiv(k, st.Lp) * Lp;
        const unsigned s0 = g * C + m * Lp + k1;
        double ar = 0.0, ai = 0.0;
        unsigned e = 0;
        for (unsigned t = 0; t < p; ++t) {
            const float2 a = src[s0 + t * cp];
            const float2 w = twv<INV>(T, e * M);
            ar += (double)a.x * (double)w.x - (double)a.y * (double)w.y;
            ai += (double)a.x * (double)w.y + (double)a.y * (double)w.x;
            e += k;
            if (e >= L) e -= L;
        }
        dst[o] = float2{(float)ar, (float)ai};
    }
}

__device__ __forceinline__ Stage stage_of(const Plan &plan, int s) {
    return Stage{plan.p[s], FDiv{plan.m[0][s], plan.l[0][s]}, FDiv{plan.m[1][s], plan.l[1][s]},
                 FDiv{plan.m[2][s], plan.l[2][s]}};
}

// the plan's stages over the first G rows of x0 (caller synchronised
// before); returns the buffer holding the natural-order result
template <int NT, bool INV>
__device__ __forceinline__ float2 *run_stages(float2 *x0, float2 *x1, const Tw &T, const Plan &plan, unsigned G,
                                              int ns) {
    // C passes through an empty asm statement per stage: what the six radix
    // variants derive from C alone (roots, twiddle indices) is then computed
    // in the stage that uses it instead of being hoisted out of the loops,
    // where it held ~100 registers live (and spilled)
    unsigned Lp = 1;
    float2 *a = x0, *b = x1;
    for (int s = 0; s < ns; ++s) {
        unsigned C = (unsigned)plan.C;
        asm volatile("" : "+s"(C));
        const Stage st = stage_of(plan, s);
        const unsigned p = (unsigned)st.p;
        switch (p) {
        case 2: stage_small<2, NT, INV>(a, b, T, C, G, Lp, st); break;
        case 3: stage_small<3, NT, INV>(a, b, T, C, G, Lp, st); break;
        case 4: stage_small<4, NT, INV>(a, b, T, C, G, Lp, st); break;
        case 5: stage_small<5, NT, INV>(a, b, T, C, G, Lp, st); break;
        case 7: stage_small<7, NT, INV>(a, b, T, C, G, Lp, st); break;
        case 8: stage_small<8, NT, INV>(a, b, T, C, G, Lp, st); break;
        default: stage_any<NT, INV>(a, b, T, C, G, Lp, p, st, plan.dC); break;
        }
        lds_sync();
        float2 *t = a;
        a = b;
        b = t;
        Lp *= p;
    }
    return a;
}

// Row-group loads into registers, element e = t + i NT of the group (row
// e / C, sample e mod C): coalesced, and in flight while the previous group's
// stages run.  Elements past the group's n rows read as zero.
template <int NT, int MAXE>
__device__ __forceinline__ void load_rows(float2 (&pf)[MAXE], const float2 *__restrict__ base, unsigned stride,
                                          unsigned C, FDiv dC, unsigned n) {
    const unsigned ne = n * C;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
        const unsigned e = tid_here() + i * NT;
        pf[i] = float2{0.f, 0.f};
        if (e < ne) {
            const unsigned g = fdiv(e, dC);
            pf[i] = base[g * stride + (e - g * C)];
        }
    }
}

// Input row i at in + (i / in_rb) * in_bstride + (i % in_rb) * in_stride +
// in_off (in_rb = nrows: one uniform stride; else e.g. the pilot rows of a
// batch of frames), output row i at out + i * out_stride + out_off.
template <int NT, int MAXE>
__device__ __forceinline__ void load_rows_b(float2 (&pf)[MAXE], const float2 *__restrict__ in, long long row0,
                                            long long stride, long long rb, long long bstride, unsigned C,
                                            FDiv dC, unsigned n) {
    const unsigned ne = n * C;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
        const unsigned e = tid_here() + i * NT;
        pf[i] = float2{0.f, 0.f};
        if (e < ne) {
            const unsigned g = fdiv(e, dC);
            const long long row = row0 + g, b = row / rb;
            pf[i] = in[b * bstride + (row - b * rb) * stride + (e - g * C)];
        }
    }
}

template <int CAP, bool INV, int NT = nt_of(CAP)>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(wpe_of(CAP), wpe_of(CAP))))
k_fft_any(const float2 *__restrict__ in, long long in_stride, long long in_rb, long long in_bstride, int in_off,
          float2 *out, long long out_stride, int out_off, long long nrows, float scale, Plan plan) {
    constexpr int MAXE = CAP / NT;
    __shared__ float2 x0[CAP], x1[CAP], lo[TLO], hi[THI];
    const unsigned C = (unsigned)plan.C, G = (unsigned)plan.G;
    fill_tables<NT>(lo, hi, C);
    const Tw T{lo, hi};
    const long long ngroups = (nrows + G - 1) / G;
    auto rows_of = [&](long long grp) { return (unsigned)(nrows - grp * G < G ? nrows - grp * G : G); };
    in += in_off;
    float2 pf[MAXE];
    long long grp = blockIdx.x;
    if (grp < ngroups) load_rows_b<NT, MAXE>(pf, in, grp * G, in_stride, in_rb, in_bstride, C, plan.dC, rows_of(grp));
    for (; grp < ngroups; grp += gridDim.x) {
        const unsigned n = rows_of(grp);
#pragma unroll
        for (int i = 0; i < MAXE; ++i) x0[tid_here() + i * NT] = pf[i];
        lds_sync();
        const long long nxt = grp + gridDim.x;
        if (nxt < ngroups) load_rows_b<NT, MAXE>(pf, in, nxt * G, in_stride, in_rb, in_bstride, C, plan.dC, rows_of(nxt));
        const float2 *res = run_stages<NT, INV>(x0, x1, T, plan, n, plan.ns);
        float2 *dst = out + grp * G * out_stride + out_off;
        for (unsigned e = tid_here(); e < n * C; e += NT) {
            const unsigned g = fdiv(e, plan.dC);
            const float2 v = res[e];
            dst[g * out_stride + (e - g * C)] = float2{v.x * scale, v.y * scale};
        }
        lds_sync();  // the next group's rows go into x0
    }
}

// The last FFT stage fused with the combine: the stage's butterfly k1 (of
// cp = C / P; Lp = cp, no output permutation left) yields bins k1 + cp k2,
// k2 < P, of one row; each is multiplied by its channel estimate (bin-layout
// Hc row, read through L2) and added to the thread's accumulator of that bin.
// A thread owns the butterflies k1 = t + j NT of every row, so its bins are
// the same for every row group of every symbol.  Rows in order, as
// matrixMultThenSum (cpuLS.hpp:187-208).
template <int P, int NT, int NACC>
__device__ __forceinline__ void last_mac(const float2 *src, const Tw &T, unsigned C, unsigned n,
                                         const float2 *__restrict__ H, float2 (&acc)[NACC]) {
    constexpr int MAXJ = NACC / P;
    const unsigned cp = C / P;
    float2 r[P];
#pragma unroll
    for (int j = 0; j < P; ++j) r[j] = (P == 3 || P == 5 || P == 7) ? twv<false>(T, j * cp) : float2{1.f, 0.f};
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        const unsigned k1 = tid_here() + j * NT;
        if (k1 < cp) {
            for (unsigned g = 0; g < n; ++g) {
                float2 a[P], h[P];
#pragma unroll
                for (int t = 0; t < P; ++t) {
                    a[t] = src[g * C + k1 + t * cp];
                    h[t] = H[g * C + k1 + t * cp];
                }
                if (k1 != 0) twiddle_powers<P, false>(a, T, k1);
                dft_small<P, false>(a, r);
#pragma unroll
                for (int k2 = 0; k2 < P; ++k2) {
                    pk::v2f z = pk::V(acc[j * P + k2]);
                    pk::mac(z, pk::V(a[k2]), pk::V(h[k2]));
                    acc[j * P + k2] = pk::F(z);
                }
            }
        }
    }
}

// ... for a last radix above 7 (a prime): one bin o = t + j NT per slot,
// out = sum_t W_C^{(t o) mod C} y[o mod cp + t cp] (double accumulation)
template <int NT, int NACC>
__device__ __forceinline__ void last_mac_any(const float2 *src, const Tw &T, unsigned C, unsigned n, unsigned p,
                                             const float2 *__restrict__ H, float2 (&acc)[NACC]) {
    const unsigned cp = C / p;
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
        const unsigned o = tid_here() + j * NT;
        if (o < C) {
            const unsigned k1 = o % cp;
            for (unsigned g = 0; g < n; ++g) {
                double ar = 0.0, ai = 0.0;
                unsigned e = 0;
                for (unsigned t = 0; t < p; ++t) {
                    const float2 a = src[g * C + k1 + t * cp];
                    const float2 w = twv<false>(T, e);
                    ar += (double)a.x * (double)w.x - (double)a.y * (double)w.y;
                    ai += (double)a.x * (double)w.y + (double)a.y * (double)w.x;
                    e += o;
                    if (e >= C) e -= C;
                }
                const float2 v{(float)ar, (float)ai}, h = H[g * C + o];
                acc[j] = float2{acc[j].x + (v.x * h.x - v.y * h.y), acc[j].y + (v.x * h.y + v.y * h.x)};
            }
        }
    }
}

// bin of accumulator slot i (last radix P; P = 0: last_mac_any's slots)
template <int P, int NT>
__device__ __forceinline__ unsigned acc_bin(int i, unsigned C) {
    if constexpr (P == 0) {
        return tid_here() + i * NT;
    } else {
        const unsigned cp = C / P, k1 = tid_here() + (i / P) * NT;
        return k1 < cp ? k1 + cp * (i % P) : ~0u;
    }
}

// a finished symbol: normalise by P and rotate, or the numerator; clears acc
template <int P, int NT, int NACC>
__device__ __forceinline__ void store_acc(float2 (&acc)[NACC], float2 *__restrict__ o, const float *__restrict__ Pf,
                                          unsigned C, int mode) {
    const unsigned K = C - 1;
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
        const unsigned b = acc_bin<P, NT>(i, C);
        if (b >= 1 && b < C) {
            const float2 a = acc[i];
            if (mode == 0) {
                const float p = Pf[b];
                o[out_pos_any((int)b - 1, (int)K)] = float2{a.x * __builtin_amdgcn_rcpf(p), a.y * __builtin_amdgcn_rcpf(p)};
            } else {
                o[b - 1] = a;
            }
        }
        acc[i] = float2{0.f, 0.f};
    }
}

// Fused any-C MRC (FFT + combine in one HBM pass): each workgroup walks data
// symbols q = blockIdx + k gridDim; per symbol the R antenna rows in groups
// of G: the group's rows (prefetched into registers during the previous
// group) go to LDS, the plan's FFT stages but the last run there, and the
// last one runs fused with the combine (last_mac).  At the end of a symbol:
// normalise by P and rotate (cpuLS.hpp:364-368, shiftOneRow's memmoves for
// any K), or store the numerator (mode 1, antenna split).  HBM traffic: the IQ
// once and the outputs; Hc and P from L2.
template <int CAP, int NT = nt_of(CAP)>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(wpe_mrc(CAP), wpe_mrc(CAP))))
k_mrc_any(const float2 *__restrict__ iq, long long nframes, int S, int R, int prefix, const float2 *__restrict__ Hc,
          const float *__restrict__ P, float2 *__restrict__ out, int mode, Plan plan) {
    constexpr int MAXE = CAP / NT;
    constexpr int NACC = MAXE + 8;  // bins per thread: ceil(C/P / NT) * P <= MAXE + P - 1
    __shared__ float2 x0[CAP], x1[CAP], lo[TLO], hi[THI];
    const unsigned C = (unsigned)plan.C, G = (unsigned)plan.G, K = C - 1;
    const unsigned Cp = C + (unsigned)prefix;
    const int PL = plan.p[plan.ns - 1];
    fill_tables<NT>(lo, hi, C);
    const Tw T{lo, hi};
    const int nsd = S - 1, ngr = (R + (int)G - 1) / (int)G;
    const long long nq = nframes * nsd;
    const long long sym_elems = (long long)R * Cp;  // one symbol of the IQ
    // work item (q, gi): data symbol q = f * nsd + (s - 1), antenna group gi;
    // frame and symbol kept as counters (no 64-bit divisions in the loop)
    long long q = blockIdx.x, f = q / nsd;
    int s = 1 + (int)(q - f * nsd), gi = 0;
    auto rows_in = [&](int g) { return (unsigned)(R - g * (int)G < (int)G ? R - g * (int)G : (int)G); };
    auto xb = [&](long long ff, int ss, int g) { return iq + (ff * S + ss) * sym_elems + (long long)g * G * Cp + prefix; };
    float2 pf[MAXE], acc[NACC];
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = float2{0.f, 0.f};
    if (q < nq) load_rows<NT, MAXE>(pf, xb(f, s, 0), Cp, C, plan.dC, rows_in(0));
    while (q < nq) {
        const unsigned n = rows_in(gi);
#pragma unroll
        for (int i = 0; i < MAXE; ++i) x0[tid_here() + i * NT] = pf[i];
        lds_sync();
        long long qn = q, fn = f;
        int sn = s, gn = gi + 1;
        if (gn == ngr) {
            gn = 0;
            qn = q + gridDim.x;
            const int t = s - 1 + (int)gridDim.x;  // symbol steps advance q by gridDim
            fn = f + t / nsd;
            sn = 1 + t % nsd;
        }
        if (qn < nq) load_rows<NT, MAXE>(pf, xb(fn, sn, gn), Cp, C, plan.dC, rows_in(gn));
        const float2 *y = run_stages<NT, false>(x0, x1, T, plan, n, plan.ns - 1);
        const float2 *H = Hc + (f * R + (long long)gi * G) * C;
        int pl = PL;
        unsigned Cl = C;
        asm volatile("" : "+s"(pl), "+s"(Cl));  // as below: nothing of the cases hoisted
        switch (pl) {
        case 2: last_mac<2, NT>(y, T, Cl, n, H, acc); break;
        case 3: last_mac<3, NT>(y, T, Cl, n, H, acc); break;
        case 4: last_mac<4, NT>(y, T, Cl, n, H, acc); break;
        case 5: last_mac<5, NT>(y, T, Cl, n, H, acc); break;
        case 7: last_mac<7, NT>(y, T, Cl, n, H, acc); break;
        case 8: last_mac<8, NT>(y, T, Cl, n, H, acc); break;
        default: last_mac_any<NT>(y, T, Cl, n, (unsigned)pl, H, acc); break;
        }
        lds_sync();  // the next group's rows go into x0
        if (gn == 0) {    // symbol q complete
            float2 *o = out + q * K;
            const float *Pf = P + f * C;
            // C and the radix pass through an empty asm statement: the store
            // indices (out_pos_any of every slot, per radix case) are then
            // computed here, not hoisted out of the loop (hundreds of
            // registers live, spilled)
            int pl2 = PL;
            unsigned Cs = C;
            asm volatile("" : "+s"(pl2), "+s"(Cs));
            switch (pl2) {
            case 2: store_acc<2, NT>(acc, o, Pf, Cs, mode); break;
            case 3: store_acc<3, NT>(acc, o, Pf, Cs, mode); break;
            case 4: store_acc<4, NT>(acc, o, Pf, Cs, mode); break;
            case 5: store_acc<5, NT>(acc, o, Pf, Cs, mode); break;
            case 7: store_acc<7, NT>(acc, o, Pf, Cs, mode); break;
            case 8: store_acc<8, NT>(acc, o, Pf, Cs, mode); break;
            default: store_acc<0, NT>(acc, o, Pf, Cs, mode); break;
            }
        }
        q = qn;
        f = fn;
        s = sn;
        gi = gn;
    }
}

// Radices in stage order: primes above 8 first (their direct stages are
// the slowest; never the fused last stage), then 8s, 7, 5, 4, 3, 2 -- the
// smallest last, so that the fused last stage of k_mrc_any has the most
// butterflies (C / p_last) to spread over the threads; a pure power of 8
// ends in 4 x 2 instead of 8 for the same reason.
bool make_plan(int C, Plan &pl) {
    if (C < 2 || C > FFT_ANY_MAX) return false;
    pl.C = C;
    pl.G = cap_of(C) / C;
    pl.ns = 0;
    pl.dC = make_fdiv((unsigned)C);
    int f[32], nf = 0, n = C;
    int c2 = 0, c3 = 0, c5 = 0, c7 = 0;
    while (n % 2 == 0) { n /= 2; ++c2; }
    while (n % 3 == 0) { n /= 3; ++c3; }
    while (n % 5 == 0) { n /= 5; ++c5; }
    while (n % 7 == 0) { n /= 7; ++c7; }
    int big[16], nbig = 0;  // prime factors above 7
    for (int p = 11; n > 1; p += 2) {
        if (p * p > n) p = n;
        while (n % p == 0) {
            if (nbig == 16) return false;
            big[nbig++] = p;
            n /= p;
        }
    }
    for (int i = 0; i < nbig; ++i) f[nf++] = big[i];
    int tail2 = 0;  // radices 4 / 2 that follow the 8s
    if (c2 % 3 == 0 && c2 > 0 && c3 + c5 + c7 == 0) {  // pure power of 8 beside primes > 8 only
        for (int i = 0; i < c2 / 3 - 1; ++i) f[nf++] = 8;
        tail2 = 3;
    } else {
        for (int i = 0; i < c2 / 3; ++i) f[nf++] = 8;
        tail2 = c2 % 3;
    }
    for (int i = 0; i < c7; ++i) f[nf++] = 7;
    for (int i = 0; i < c5; ++i) f[nf++] = 5;
    if (tail2 == 2) f[nf++] = 4;
    if (tail2 == 3) f[nf++] = 4;
    for (int i = 0; i < c3; ++i) f[nf++] = 3;
    if (tail2 == 1 || tail2 == 3) f[nf++] = 2;
    if (nf > MAX_STAGES) return false;
    int Lp = 1;
    for (int i = 0; i < nf; ++i) {
        const int p = f[i];
        const FDiv d[3] = {make_fdiv((unsigned)(C / p)), make_fdiv((unsigned)Lp), make_fdiv((unsigned)(Lp * p))};
        for (int k = 0; k < 3; ++k) {
            pl.m[k][pl.ns] = d[k].m;
            pl.l[k][pl.ns] = d[k].l;
        }
        pl.p[pl.ns++] = p;
        Lp *= p;
    }
    return true;
}

// resident workgroups of a variant (LDS and registers): 4 per CU at CAP 2048,
// 2 at 4096, 1 at 8192
int resident(int cap) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return (cap == 2048 ? 4 : cap == 4096 ? 2 : 1) * cus;
}

template <int CAP>
hipError_t launch_t(const float2 *in, long long in_stride, long long in_rb, long long in_bstride, int in_off,
                    float2 *out, long long out_stride, int out_off, long long nrows, bool inverse, float scale,
                    const Plan &pl, hipStream_t s) {
    const long long groups = (nrows + pl.G - 1) / pl.G;
    const long long res = resident(CAP);
    const unsigned grid = (unsigned)(groups < res ? groups : res);  // persistent over the row groups
    if (inverse)
        hipLaunchKernelGGL((k_fft_any<CAP, true>), dim3(grid), dim3(nt_of(CAP)), 0, s, in, in_stride, in_rb,
                           in_bstride, in_off, out, out_stride, out_off, nrows, scale, pl);
    else
        hipLaunchKernelGGL((k_fft_any<CAP, false>), dim3(grid), dim3(nt_of(CAP)), 0, s, in, in_stride, in_rb,
                           in_bstride, in_off, out, out_stride, out_off, nrows, scale, pl);
    return hipGetLastError();
}

template <int CAP>
hipError_t launch_mrc_t(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hc,
                        const float *P, float2 *out, int mode, const Plan &pl, hipStream_t s) {
    const long long nq = nframes * (S - 1);
    const long long res = resident(CAP) / (CAP == 2048 ? 4 : 1) * (CAP == 2048 ? 3 : 1);
    const unsigned grid = (unsigned)(nq < res ? nq : res);  // persistent: one round of resident workgroups
    hipLaunchKernelGGL((k_mrc_any<CAP>), dim3(grid), dim3(nt_of(CAP)), 0, s, iq, nframes, S, R, prefix, Hc, P, out,
                       mode, pl);
    return hipGetLastError();
}

}  // namespace fany

bool fft_any_supported(int C) {
    fany::Plan pl;
    return fany::make_plan(C, pl);
}

hipError_t launch_fft_any_b(const float2 *in, long long in_stride, long long in_rb, long long in_bstride,
                            int in_off, float2 *out, long long out_stride, int out_off, long long nrows, int C,
                            bool inverse, float scale, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    fany::Plan pl;
    if (!fany::make_plan(C, pl) || in_rb < 1) return hipErrorInvalidValue;
#define OFDM_FANY(CAP) \
    fany::launch_t<CAP>(in, in_stride, in_rb, in_bstride, in_off, out, out_stride, out_off, nrows, inverse, scale, pl, s)
    switch (fany::cap_of(C)) {
    case 2048: return OFDM_FANY(2048);
    case 4096: return OFDM_FANY(4096);
    default: return OFDM_FANY(8192);
    }
#undef OFDM_FANY
}

hipError_t launch_fft_any(const float2 *in, long long in_stride, int in_off, float2 *out, long long out_stride,
                          int out_off, long long nrows, int C, bool inverse, float scale, hipStream_t s) {
    return launch_fft_any_b(in, in_stride, nrows > 0 ? nrows : 1, 0, in_off, out, out_stride, out_off, nrows, C,
                            inverse, scale, s);
}

hipError_t launch_mrc_any(const float2 *iq, long long nframes, int S, int R, int C, int prefix, const float2 *Hc,
                          const float *P, float2 *out, int mode, hipStream_t s) {
    if (nframes <= 0 || S < 2) return hipSuccess;
    fany::Plan pl;
    if (!fany::make_plan(C, pl)) return hipErrorInvalidValue;
    switch (fany::cap_of(C)) {
    case 2048: return fany::launch_mrc_t<2048>(iq, nframes, S, R, prefix, Hc, P, out, mode, pl, s);
    case 4096: return fany::launch_mrc_t<4096>(iq, nframes, S, R, prefix, Hc, P, out, mode, pl, s);
    default: return fany::launch_mrc_t<8192>(iq, nframes, S, R, prefix, Hc, P, out, mode, pl, s);
    }
}

}  // namespace ofdm
