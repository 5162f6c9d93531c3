// zf.hip -- multi-user zero-forcing on the GPU:
// the reference's precoder createZeroForcingMatrix (cpuLS.hpp:415-447:
// rotCube, per-subcarrier cgemm A A^H, cgetrf + cgetri, cgemm A^H G^-1),
// multiplyWithChannelInv (449-463, per-subcarrier cgemv) and the uplink
// counterpart, ZF detection with the same matrix.
//
// Per subcarrier k the shapes are small (users U <= 32, antennas R,
// U*R <= 8192): G = A A^H is U x U x R, the inverse U^3, W = A^H G^-1 is
// R x U x U.  One 1023-subcarrier channel set at U = 16, R = 64 is ~0.3 GFLOP
// -- a few microseconds of VALU next to ~16 MB of HBM traffic.
//   k_zf_precoder: one 256-thread workgroup per subcarrier; A (U x R) and G
//     in LDS; LU with partial pivoting (pivot = first max of |re| + |im|,
//     LAPACK's icamax in cgetrf) and the inverse in cgetri's order, with no
//     fused multiply-adds -- bit-identical to the oracle.  W is written in
//     the reference's layout W[k][u][r] (per subcarrier R x U column-major)
//     and/or the subcarrier-fastest layout Wt[u][r][k] the apply / detect
//     kernels read with coalesced loads.
//   k_zf_gemm: the symbol-batched application -- for every subcarrier a small
//     complex GEMM out_k (M x nsym) = A_k (M x N) . in_k (N x nsym), A_k = W
//     (apply: M = R, N = U) or W^H (detect: M = U, N = R).  Lanes = 64
//     consecutive subcarriers (the fastest axis of every operand, so each load
//     and store is one coalesced 512 B wave access); each wave accumulates an
//     MT x ST (rows x symbols) register tile, so per n it loads MT + ST values
//     for MT * ST complex MACs.  At U = 16, R = 64 the work is ~13 flop per HBM
//     byte, under the FP32 ridge (~20): HBM-bound on paper (at U = 32, 26
//     flop/B, compute-bound).  The f32 matrix peak of gfx950 equals its f32
//     vector peak (MI355X_MICROARCH.md); the k_zf_mfma_* / k_zf_wstat kernels
//     below put the MACs on the matrix cores anyway (16-block 4x4x1 MFMA, one
//     block per subcarrier) and win for detect at U > 8.
//     The W tile of a (subcarrier block, row block) is re-read for every symbol
//     step; block ids are mapped so that all workgroups of one XCD share the
//     same few tiles (dispatch is round-robin over the 8 XCDs), keeping those
//     re-reads in that XCD's 4 MB L2 instead of HBM.
#include <hip/hip_runtime.h>

#include "launch.hpp"
#include "pk.hpp"

namespace ofdm {
namespace zf {

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return float2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // conj(a) * b
    return float2{a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float cabs1(float2 a) { return fabsf(a.x) + fabsf(a.y); }
__device__ __forceinline__ float2 crcp(float2 a) {  // 1 / a
    const float d = a.x * a.x + a.y * a.y;
    return float2{a.x / d, -a.y / d};
}

constexpr int MAXU = 32;

// 1 / a by Smith's algorithm (what LAPACK's ONE / A(J,J) compiles to under
// gfortran's complex-division rules): the oracle (oracle/zf_oracle.c) uses
// the same formula, so with contraction off the precoder is bit-identical.
__device__ __forceinline__ float2 crcp_smith(float2 a) {
#pragma clang fp contract(off)
    if (fabsf(a.x) >= fabsf(a.y)) {
        const float r = a.y / a.x, den = a.x + a.y * r;
        return float2{1.f / den, -r / den};
    }
    const float r = a.x / a.y, den = a.x * r + a.y;
    return float2{r / den, -1.f / den};
}
__device__ __forceinline__ float2 cmul_nc(float2 a, float2 b) {  // a * b, no contraction
#pragma clang fp contract(off)
    return float2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

// One 256-thread workgroup per subcarrier.  G = A A^H, its LU factors with
// partial pivoting (LAPACK cgetf2: pivot = first max of |re| + |im|), the
// inverse from them as cgetri computes it (ctrti2 on U, then inv(A) L =
// inv(U) column by column from the right, then the column interchanges), and
// W = A^H G^-1 -- every element accumulated in the oracle's order with no
// fused multiply-adds, the independent elements of each step in parallel.
__global__ void __launch_bounds__(256) k_zf_precoder(const float2 *__restrict__ Hin, int U, int R, int K,
                                                     float2 *__restrict__ W, float2 *__restrict__ Wt) {
#pragma clang fp contract(off)
    extern __shared__ float2 sm[];
    float2 *A = sm;          // A(u, r) at A[r*U + u]: X[col] after rotCube (cpuLS.hpp:404-410)
    float2 *G = sm + U * R;  // U x U column-major: G(i, c) at G[c*U + i]
    __shared__ float2 col[MAXU];
    __shared__ int ipiv[MAXU];
    const int t = threadIdx.x, k = blockIdx.x, n = U;

    for (int e = t; e < U * R; e += 256) {
        const int u = e / R, r = e - u * R;
        A[r * U + u] = Hin[((long long)u * R + r) * K + k];
    }
    __syncthreads();
    // G(a, b) = sum_r A(a, r) conj(A(b, r))   (cgemm NoTrans / ConjTrans, cpuLS.hpp:437)
    for (int e = t; e < U * U; e += 256) {
        const int a = e % U, b = e / U;
        float2 s{0.f, 0.f};
        for (int r = 0; r < R; ++r) {
            const float2 x = A[r * U + a], y = A[r * U + b];
            s.x = s.x + (x.x * y.x + x.y * y.y);
            s.y = s.y + (x.y * y.x - x.x * y.y);
        }
        G[b * n + a] = s;
    }
    __syncthreads();
    // cgetrf (unblocked cgetf2), cpuLS.hpp:438
    for (int j = 0; j < n; ++j) {
        if (t == 0) {
            int p = j;
            for (int i = j + 1; i < n; ++i)
                if (cabs1(G[j * n + i]) > cabs1(G[j * n + p])) p = i;
            ipiv[j] = p;
        }
        __syncthreads();
        const int p = ipiv[j];
        const float2 gp = G[j * n + p];
        const bool nz = gp.x != 0.f || gp.y != 0.f;
        if (nz && p != j)
            for (int c = t; c < n; c += 256) {
                const float2 tmp = G[c * n + j];
                G[c * n + j] = G[c * n + p];
                G[c * n + p] = tmp;
            }
        __syncthreads();
        if (nz) {
            const float2 rj = crcp_smith(G[j * n + j]);
            for (int i = j + 1 + t; i < n; i += 256) G[j * n + i] = cmul_nc(G[j * n + i], rj);
        }
        __syncthreads();
        for (int e = t; e < (n - j - 1) * (n - j - 1); e += 256) {
            const int c = j + 1 + e / (n - j - 1), i = j + 1 + e % (n - j - 1);
            const float2 m = cmul_nc(G[j * n + i], G[c * n + j]);
            G[c * n + i] = float2{G[c * n + i].x - m.x, G[c * n + i].y - m.y};
        }
        __syncthreads();
    }
    // cgetri, cpuLS.hpp:439.  ctrti2: column j of inv(U) from the inverted
    // columns 0..j-1: x(i) = orig(i,j) U^-1(i,i) + sum_{c=i+1}^{j-1} orig(c,j)
    // U^-1(i,c), then x(i) * (-U^-1(j,j))
    for (int j = 0; j < n; ++j) {
        if (t < j) col[t] = G[j * n + t];
        const float2 djj = crcp_smith(G[j * n + j]);  // read before thread 0 overwrites it
        __syncthreads();
        if (t < j) {
            float2 x = cmul_nc(col[t], G[t * n + t]);
            for (int c = t + 1; c < j; ++c) {
                const float2 m = cmul_nc(col[c], G[c * n + t]);
                x = float2{x.x + m.x, x.y + m.y};
            }
            G[j * n + t] = cmul_nc(x, float2{-djj.x, -djj.y});
        }
        if (t == 0) G[j * n + j] = djj;
        __syncthreads();
    }
    // inv(A) L = inv(U), columns right to left: column j -= sum_{c>j} col c * L(c, j)
    for (int j = n - 1; j >= 0; --j) {
        if (t > j && t < n) col[t] = G[j * n + t];
        __syncthreads();
        if (t < n) {
            float2 x = t > j ? float2{0.f, 0.f} : G[j * n + t];
            for (int c = j + 1; c < n; ++c) {
                const float2 m = cmul_nc(G[c * n + t], col[c]);
                x = float2{x.x - m.x, x.y - m.y};
            }
            G[j * n + t] = x;
        }
        __syncthreads();
    }
    // the row interchanges, undone as column interchanges, last first
    for (int j = n - 2; j >= 0; --j) {
        const int p = ipiv[j];
        if (p != j && t < n) {
            const float2 tmp = G[j * n + t];
            G[j * n + t] = G[p * n + t];
            G[p * n + t] = tmp;
        }
        __syncthreads();
    }
    // W(r, u) = sum_a conj(A(a, r)) Ginv(a, u)   (cgemm ConjTrans / NoTrans, cpuLS.hpp:440)
    for (int e = t; e < R * U; e += 256) {
        const int u = e / R, r = e - u * R;
        float2 s{0.f, 0.f};
        for (int a = 0; a < U; ++a) {
            const float2 x = A[r * U + a], g = G[u * n + a];
            s.x = s.x + (x.x * g.x + x.y * g.y);
            s.y = s.y + (x.x * g.y - x.y * g.x);
        }
        if (W) W[(long long)k * R * U + u * R + r] = s;
        if (Wt) Wt[((long long)u * R + r) * K + k] = s;
    }
}

// Reference layout W[k][u][r] -> Wt[u][r][k] through a 64 x 64 LDS tile
// (k block x (u,r) block); both the global read and write are coalesced.
__global__ void __launch_bounds__(256) k_zf_transpose(const float2 *__restrict__ W, int UR, int K,
                                                      float2 *__restrict__ Wt) {
    __shared__ float2 tile[64][65];
    const int k0 = blockIdx.x * 64, e0 = blockIdx.y * 64;
    const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
    for (int i = ly; i < 64; i += 4) {
        const int k = k0 + i, e = e0 + lx;
        if (k < K && e < UR) tile[i][lx] = W[(long long)k * UR + e];
    }
    __syncthreads();
    for (int i = ly; i < 64; i += 4) {
        const int e = e0 + i, k = k0 + lx;
        if (k < K && e < UR) Wt[(long long)e * K + k] = tile[lx][i];
    }
}

// out[s][m][k] = sum_n A_k(m, n) in[s][n][k],
// A_k(m, n) = Wt[(m*a_m + n*a_n)*K + k] (conjugated if CONJ).
// Workgroup = 4 waves = MG row groups x (4/MG) symbol groups; it owns the
// rows [mb*MG*MT, +MG*MT) of a 64-subcarrier block and walks its symbol chunk
// in steps of (4/MG)*ST symbols.
// PF: the loads of step n+1 are issued before the MACs of step n (register
// double buffering), so a wave's memory latency overlaps its own arithmetic.
template <int MT, int ST, int MG, bool CONJ, bool PF>
__global__ void __launch_bounds__(256) k_zf_gemm(const float2 *__restrict__ Wt, int a_m, int a_n,
                                                 const float2 *__restrict__ in, int N, int M, int K,
                                                 long long nsym, float2 *__restrict__ out, int ntile,
                                                 int tpx, int nkb, long long chunk_steps) {
    constexpr int SG = 4 / MG, SBLK = SG * ST;
    // XCD-aware block mapping: block b runs on XCD b % 8; XCD x owns tiles
    // x, x+8, x+16, ... and walks all symbol chunks of them.
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    const int tile = xcd + 8 * (j % tpx);
    if (tile >= ntile) return;
    const long long chunk = j / tpx;
    const int kb = tile % nkb, mb = tile / nkb;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int k = kb * 64 + lane;
    if (k >= K) return;  // no barriers below
    const int m0 = (mb * MG + (w % MG)) * MT;
    if (m0 >= M) return;
    const long long step0 = chunk * chunk_steps;
    const long long nsteps_total = (nsym + SBLK - 1) / SBLK;
    const long long step1 = min(step0 + chunk_steps, nsteps_total);

    // one 64-bit base per operand; row / symbol offsets are wave-uniform ints
    // (clamped to the last valid row / symbol: those lanes compute, never store)
    const float2 *wb = Wt + (long long)m0 * a_m * K + k;
    const int amK = a_m * K, anK = a_n * K, NK = N * K, mlast = M - 1 - m0;

    for (long long st = step0; st < step1; ++st) {
        const long long s0 = st * SBLK + (w / MG) * ST;
        const int slast = (int)min((long long)ST - 1, nsym - 1 - s0);
        const float2 *xb = in + s0 * NK + k;
        float2 acc[MT][ST];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int jj = 0; jj < ST; ++jj) acc[i][jj] = float2{0.f, 0.f};
        float2 a[MT], x[ST];
        auto load = [&](int n, float2 *av, float2 *xv) {
            const float2 *wn = wb + n * anK, *xn = xb + n * K;
#pragma unroll
            for (int i = 0; i < MT; ++i) av[i] = wn[min(i, mlast) * amK];
#pragma unroll
            for (int jj = 0; jj < ST; ++jj) xv[jj] = xn[min(jj, slast) * NK];
        };
        if (PF) load(0, a, x);
#pragma unroll 2
        for (int n = 0; n < N; ++n) {
            float2 an[MT], xnx[ST];
            if (PF)
                load(min(n + 1, N - 1), an, xnx);  // the last one is a redundant reload
            else
                load(n, a, x);
            // complex MAC as 4 FMAs straight into the accumulator
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const float ar = a[i].x, ai = CONJ ? -a[i].y : a[i].y;
#pragma unroll
                for (int jj = 0; jj < ST; ++jj) {
                    acc[i][jj].x = fmaf(ar, x[jj].x, fmaf(-ai, x[jj].y, acc[i][jj].x));
                    acc[i][jj].y = fmaf(ar, x[jj].y, fmaf(ai, x[jj].x, acc[i][jj].y));
                }
            }
            if (PF) {
#pragma unroll
                for (int i = 0; i < MT; ++i) a[i] = an[i];
#pragma unroll
                for (int jj = 0; jj < ST; ++jj) x[jj] = xnx[jj];
            }
        }
#pragma unroll
        for (int jj = 0; jj < ST; ++jj) {
            if (s0 + jj >= nsym) break;
            float2 *o = out + ((s0 + jj) * M) * (long long)K + k;
#pragma unroll
            for (int i = 0; i < MT; ++i)
                if (m0 + i < M) o[(long long)(m0 + i) * K] = acc[i][jj];
        }
    }
}

// The same GEMM with the operand tiles shared through LDS (default for M > 4,
// N >= 8).
// Each wave of k_zf_gemm loads its own 8 + 8 operand rows per n, so at U = 16
// the per-CU L1 path (64 B/clk) had to carry twice the unique bytes and capped
// the kernel at ~37 % of HBM.  Here the workgroup stages each chunk of NC
// n-steps -- the MB = MG*8 rows of A and the SB = (4/MG)*8 symbols of the
// input, 64 subcarriers each -- once, with plain coalesced loads into
// registers, and every wave reads its 8 + 8 rows per n from LDS (128 B/clk,
// conflict free: 64 lanes x 8 B contiguous).  The loads of chunk c+1 are in
// flight while chunk c is computed; two LDS buffers, one barrier per chunk.
// ST = 4, NC = 1 (OFDM_ZF_ST=4): 8x4 tiles, 64 accumulator VGPRs, 4 waves/SIMD.
// XMAP (OFDM_ZF_XMAP=1): XCD x takes symbol chunks x, x + 8, ... with all
// tiles (the k_zf_wstat map) instead of tiles x, x + 8, ... with all chunks.
template <int MG, bool CONJ, bool NTIN = false, int ST = 8, int NC = 2, bool XMAP = false>
__global__ void __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(ST == 4 ? 4 : 1)))
k_zf_gemm_lds(const float2 *__restrict__ Wt, int a_m, int a_n, const float2 *__restrict__ in, int N, int M,
              int K, long long nsym, float2 *__restrict__ out, int ntile, int tpx, int nkb,
              long long chunk_steps) {
    constexpr int MT = 8, SG = 4 / MG, MB = MG * MT, SB = SG * ST;
    constexpr int AROWS = NC * MB, ROWS = NC * (MB + SB), RPT = ROWS / 4, AI = AROWS / 4;
    static_assert(AROWS % 4 == 0 && ROWS % 4 == 0, "rows split evenly over the 4 waves");
    __shared__ float2 sm[2][ROWS * 64];
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;  // XCD-aware mapping as k_zf_gemm
    const int tile = XMAP ? j % ntile : xcd + 8 * (j % tpx);
    if (tile >= ntile) return;  // whole workgroup
    const long long chunk = XMAP ? xcd + 8LL * (j / ntile) : j / tpx;
    const int kb = tile % nkb, mb = tile / nkb;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int k = kb * 64 + lane, kc = min(k, K - 1);  // lanes past K load a valid bin, never store
    const int mg = w % MG, sg = w / MG, mb0 = mb * MB;
    const long long nsteps_total = (nsym + SB - 1) / SB;
    const long long step0 = chunk * chunk_steps, step1 = min(step0 + chunk_steps, nsteps_total);
    const int nnc = (N + NC - 1) / NC;
    const long long nseq = (step1 - step0) * nnc;
    if (nseq <= 0) return;  // whole workgroup

    // chunk c = (symbol step cs, n-chunk cn), walked with int counters: a
    // 64-bit c / nnc per chunk made the loop SALU-bound (22 k scalar
    // instructions per wave against 40 k VALU at U = 16)
    float2 stg[RPT];
    // per-row element offsets of the in-range fast path, relative to the
    // chunk's n0 (A rows) / (s0, n0) (input rows): wave-uniform, loop-invariant
    int roff[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int row = w + 4 * i;
        if (i < AI)
            roff[i] = (min(mb0 + row % MB, M - 1) * a_m + (row / MB) * a_n) * K;
        else
            roff[i] = (((row - AROWS) % SB) * N + (row - AROWS) / SB) * K;
    }
    auto load = [&](int cs, int cn) {
        const long long s0 = (step0 + cs) * SB;
        const int n0 = cn * NC;
        if (n0 + NC <= N && s0 + SB <= nsym) {  // whole chunk in range: one 64-bit base per operand
            const float2 *pa = Wt + (long long)n0 * a_n * K + kc;
            const float2 *px = in + (s0 * N + n0) * (long long)K + kc;
#pragma unroll
            for (int i = 0; i < RPT; ++i) {
                if (i < AI) {
                    stg[i] = pa[roff[i]];
                } else if constexpr (NTIN) {
                    stg[i] = __builtin_bit_cast(float2, __builtin_nontemporal_load(
                                                            reinterpret_cast<const unsigned long long *>(px + roff[i])));
                } else {
                    stg[i] = px[roff[i]];
                }
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int row = w + 4 * i;
            if (i < AI) {  // A rows: (n, m) = (n0 + row / MB, mb0 + row % MB)
                const int n = min(n0 + row / MB, N - 1), m = min(mb0 + row % MB, M - 1);
                stg[i] = Wt[((long long)m * a_m + (long long)n * a_n) * K + kc];
            } else {  // input rows: (n, s) = (n0 + rr / SB, s0 + rr % SB)
                const int rr = row - AROWS;
                const int n = min(n0 + rr / SB, N - 1);
                const long long s = min(s0 + rr % SB, nsym - 1);
                const float2 *p = in + (s * N + n) * (long long)K + kc;
                if constexpr (NTIN)  // streamed once: keep it from evicting the re-read W tiles
                    stg[i] = __builtin_bit_cast(
                        float2, __builtin_nontemporal_load(reinterpret_cast<const unsigned long long *>(p)));
                else
                    stg[i] = *p;
            }
        }
    };
    auto put = [&](int buf) {
#pragma unroll
        for (int i = 0; i < RPT; ++i) sm[buf][(w + 4 * i) * 64 + lane] = stg[i];
    };

    float2 acc[MT][ST];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jj = 0; jj < ST; ++jj) acc[i][jj] = float2{0.f, 0.f};
    load(0, 0);
    put(0);
    __syncthreads();
    const int nst = (int)(step1 - step0);
    int cs = 0, cn = 0, buf = 0;
    for (;;) {
        const int ncn = cn + 1 == nnc ? 0 : cn + 1, ncs = cn + 1 == nnc ? cs + 1 : cs;
        const bool more = ncs < nst;
        if (more) load(ncs, ncn);  // in flight during this chunk's MACs
        const float2 *sa = sm[buf] + (mg * MT) * 64 + lane;
        const float2 *sx = sm[buf] + (AROWS + sg * ST) * 64 + lane;
        const int n0 = cn * NC, nn = min(NC, N - n0);
        for (int n = 0; n < nn; ++n) {
            float2 a[MT], x[ST];
#pragma unroll
            for (int i = 0; i < MT; ++i) a[i] = sa[(n * MB + i) * 64];
#pragma unroll
            for (int jj = 0; jj < ST; ++jj) x[jj] = sx[(n * SB + jj) * 64];
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const float ar = a[i].x, ai = CONJ ? -a[i].y : a[i].y;
#pragma unroll
                for (int jj = 0; jj < ST; ++jj) {
                    acc[i][jj].x = fmaf(ar, x[jj].x, fmaf(-ai, x[jj].y, acc[i][jj].x));
                    acc[i][jj].y = fmaf(ar, x[jj].y, fmaf(ai, x[jj].x, acc[i][jj].y));
                }
            }
        }
        if (cn == nnc - 1) {  // last n-chunk of a symbol step: store, reset
            const long long s0 = (step0 + cs) * SB + sg * ST;
            const int m0 = mb0 + mg * MT;
            if (k < K) {
                float2 *o = out + (s0 * M + m0) * (long long)K + k;
                if (s0 + ST <= nsym && m0 + MT <= M) {  // whole tile in range: no per-store branches
#pragma unroll
                    for (int jj = 0; jj < ST; ++jj)
#pragma unroll
                        for (int i = 0; i < MT; ++i) o[(long long)(jj * M + i) * K] = acc[i][jj];
                } else {
#pragma unroll
                    for (int jj = 0; jj < ST; ++jj) {
                        if (s0 + jj >= nsym) break;
#pragma unroll
                        for (int i = 0; i < MT; ++i)
                            if (m0 + i < M) o[(long long)(jj * M + i) * K] = acc[i][jj];
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int jj = 0; jj < ST; ++jj) acc[i][jj] = float2{0.f, 0.f};
        }
        if (!more) break;
        buf ^= 1;
        put(buf);  // that buffer was last read in the previous chunk
        cs = ncs;
        cn = ncn;
        __syncthreads();
    }
}

typedef __attribute__((address_space(3))) void lvoid_t;

// The GEMM on the matrix cores (the k_zf_mfma_* / k_zf_wstat kernels below):
// v_mfma_f32_4x4x1_16b_f32
// runs 16 INDEPENDENT 4 x 4 x 1 outer products per instruction, one per
// 4-lane block, at the full f32 matrix rate (64 flop/clk/SIMD, the f32 vector
// peak, MI355X_MICROARCH.md) -- so each block is one subcarrier and the
// subcarrier-fastest layouts need no transposition: lane l = 4 b + i works on
// subcarrier k0 + b.  Complex -> real: the 4 rows of a block are
// (re m, im m, re m+1, im m+1), its 4 columns 4 symbols; per complex n two
// MFMAs with the real k-steps Xr and Xi:
//   A(re step) = (Ar, Ai, Ar', Ai'),  A(im step) = (-Ai, Ar, -Ai', Ar')
// (Ai -> -Ai for CONJ), B = Xr or Xi of the lane's symbol.  Lane (b, i) loads
// W(m0 + 2p + i/2, n) and picks its component with one select per step; lane
// (b, j) loads x[s0 + 4g + j][n][k0 + b].  D(row i, col j) of block b sits in
// accumulator register i of lane 4 b + j: lane (b, j) stores two float2.
// Each wave owns MP row pairs x SG symbol quads of 16 subcarriers; the 4 waves
// of a workgroup take consecutive symbol quads of the same W tile (shared in
// L1); operands of n+1 are loaded before the MFMAs of n.  f32 MFMA
// accumulation is an exact f32 fma chain (MI355X_MICROARCH.md).
typedef float mf4 __attribute__((ext_vector_type(4)));

// The MFMA GEMM fed through LDS: the workgroup DMA's each n-step's operand
// rows -- MB rows of A and SB symbols of the input, 64 subcarriers (512 B)
// each, coalesced -- into one of NB = 4 LDS buffers (global_load_lds_dword:
// lane l's dword lands at LDS byte base + 4 l, so rows land in their natural
// float2 order with no VGPR staging; three steps in flight, one barrier per
// step), and each wave runs the MFMAs of its 16 subcarriers reading its
// operands from LDS.  The DMAs are inline asm on purpose: through
// __builtin_amdgcn_global_load_lds the compiler cannot tell which buffer a
// ds_read may alias and puts s_waitcnt vmcnt(0) in front of every LDS read,
// draining the prefetch; the loop's own s_waitcnt vmcnt(N) + s_barrier
// publish the data instead.  M0 is compiler-reserved: saved and restored in
// the same statement, with the s_nop the M0 write -> LDS-DMA hazard needs
// (cdna_hip_programming.md).
// The 12 dword DMAs of one wave's step in k_zf_mfma_lds8 (6 rows x 2 halves,
// row r at LDS byte lds + 4096 r, half h at + 256 h), M0 saved once.
__device__ __forceinline__ void dma_rows6(const float *const (&g)[12], unsigned lds) {
    const unsigned l0 = lds + 0u;
    const unsigned l1 = lds + 256u;
    const unsigned l2 = lds + 4096u;
    const unsigned l3 = lds + 4352u;
    const unsigned l4 = lds + 8192u;
    const unsigned l5 = lds + 8448u;
    const unsigned l6 = lds + 12288u;
    const unsigned l7 = lds + 12544u;
    const unsigned l8 = lds + 16384u;
    const unsigned l9 = lds + 16640u;
    const unsigned l10 = lds + 20480u;
    const unsigned l11 = lds + 20736u;
    unsigned keep;
    asm volatile("s_mov_b32 %[keep], m0\n\t"
                 "s_mov_b32 m0, %[l0]\n\ts_nop 0\n\tglobal_load_lds_dword %[a0], off\n\t"
                 "s_mov_b32 m0, %[l1]\n\ts_nop 0\n\tglobal_load_lds_dword %[a1], off\n\t"
                 "s_mov_b32 m0, %[l2]\n\ts_nop 0\n\tglobal_load_lds_dword %[a2], off\n\t"
                 "s_mov_b32 m0, %[l3]\n\ts_nop 0\n\tglobal_load_lds_dword %[a3], off\n\t"
                 "s_mov_b32 m0, %[l4]\n\ts_nop 0\n\tglobal_load_lds_dword %[a4], off\n\t"
                 "s_mov_b32 m0, %[l5]\n\ts_nop 0\n\tglobal_load_lds_dword %[a5], off\n\t"
                 "s_mov_b32 m0, %[l6]\n\ts_nop 0\n\tglobal_load_lds_dword %[a6], off\n\t"
                 "s_mov_b32 m0, %[l7]\n\ts_nop 0\n\tglobal_load_lds_dword %[a7], off\n\t"
                 "s_mov_b32 m0, %[l8]\n\ts_nop 0\n\tglobal_load_lds_dword %[a8], off\n\t"
                 "s_mov_b32 m0, %[l9]\n\ts_nop 0\n\tglobal_load_lds_dword %[a9], off\n\t"
                 "s_mov_b32 m0, %[l10]\n\ts_nop 0\n\tglobal_load_lds_dword %[a10], off\n\t"
                 "s_mov_b32 m0, %[l11]\n\ts_nop 0\n\tglobal_load_lds_dword %[a11], off\n\t"
                 "s_mov_b32 m0, %[keep]"
                 : [keep] "=&s"(keep)
                 : [a0] "v"(g[0]), [a1] "v"(g[1]), [a2] "v"(g[2]), [a3] "v"(g[3]), [a4] "v"(g[4]), [a5] "v"(g[5]), [a6] "v"(g[6]), [a7] "v"(g[7]), [a8] "v"(g[8]), [a9] "v"(g[9]), [a10] "v"(g[10]), [a11] "v"(g[11]),
                   [l0] "s"(l0), [l1] "s"(l1), [l2] "s"(l2), [l3] "s"(l3), [l4] "s"(l4), [l5] "s"(l5), [l6] "s"(l6), [l7] "s"(l7), [l8] "s"(l8), [l9] "s"(l9), [l10] "s"(l10), [l11] "s"(l11)
                 : "memory");
}

// The LDS-fed MFMA GEMM with 8 waves (512 threads) per workgroup: MB = 4 MPW rows of
// A and SB = 4 SG symbols per step, every wave keeping MPW x SG x 4 = 128
// accumulators so that two waves share each SIMD.  Wave w computes
// subcarriers 16 (w & 3) + b of the block for row pairs MPW (w >> 2) .. + MPW-1
// and stages rows w + 8 r of every step (the first MB / 8 of them A rows).
// <8, 4>: 32-row tiles, so at M = 32 every input row is staged once instead
// of once per 16-row block.
template <int MPW, int SG, bool CONJ>
__global__ void __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(2, 2)))
k_zf_mfma_lds8(const float2 *__restrict__ Wt, int a_m, int a_n, const float2 *__restrict__ in, int N, int M,
               int K, long long nsym, float2 *__restrict__ out, int ntile, int tpx, int nkb,
               long long chunk_steps) {
    constexpr int MP = MPW, MB = 4 * MPW, SB = 4 * SG, NB = 4;
    constexpr int ROWS = MB + SB, RPW = ROWS / 8, WR = MB / 8, LPW = 2 * RPW;
    static_assert(ROWS % 8 == 0 && RPW == 6 && (NB - 2) * LPW <= 63, "rows per wave / vmcnt range");
    extern __shared__ __attribute__((aligned(16))) float2 smd[];  // [NB][ROWS][64]
    const int bid = blockIdx.x, xcd = bid & 7, jb = bid >> 3;    // XCD-aware mapping as k_zf_gemm
    const int tile = xcd + 8 * (jb % tpx);
    if (tile >= ntile) return;  // whole workgroup
    const long long chunk = jb / tpx;
    const int kb = tile % nkb, mb = tile / nkb;
    const int lane = threadIdx.x & 63, b = lane >> 2, i = lane & 3;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sub = w & 3, half = w >> 2;
    const int k = kb * 64 + 16 * sub + b;
    const int mb0 = mb * MB, m0 = mb0 + 2 * MP * half;
    const long long nsteps_total = (nsym + SB - 1) / SB;
    const long long step0 = chunk * chunk_steps, step1 = min(step0 + chunk_steps, nsteps_total);
    if (step1 <= step0) return;  // whole workgroup
    const int nst = (int)(step1 - step0);
    const int off0 = min(kb * 64 + (lane >> 1), K - 1) * 2 + (lane & 1);
    const int off1 = min(kb * 64 + 32 + (lane >> 1), K - 1) * 2 + (lane & 1);
    const bool odd = i & 1;
    const long long anK = (long long)a_n * K, NK = (long long)N * K;

    int si = 0, ni = 0, bi = 0;
    const float *wbase[WR];
#pragma unroll
    for (int r = 0; r < WR; ++r)
        wbase[r] = reinterpret_cast<const float *>(Wt + (long long)min(mb0 + w + 8 * r, M - 1) * a_m * K);
    const unsigned lds0 = (unsigned)(size_t)(lvoid_t *)smd + (unsigned)(w * 512);
    auto issue = [&]() {
        const unsigned la = lds0 + (unsigned)(bi * ROWS * 512);
        const long long s0 = (step0 + si) * SB;
        const float *ga[2 * RPW];
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const float *src;
            if (r < WR) {
                src = wbase[r] + 2 * (ni * anK);
            } else {
                const long long s = min(s0 + (w + 8 * r - MB), nsym - 1);
                src = reinterpret_cast<const float *>(in + s * NK + (long long)ni * K);
            }
            ga[2 * r] = src + off0;
            ga[2 * r + 1] = src + off1;
        }
        dma_rows6(ga, la);
        if (si < nst - 1 || ni < N - 1) {  // advance (the tail re-issues the last step)
            if (++ni == N) {
                ni = 0;
                ++si;
            }
        }
        bi = (bi + 1) & (NB - 1);
    };

    mf4 acc[MP][SG];
#pragma unroll
    for (int p = 0; p < MP; ++p)
#pragma unroll
        for (int g = 0; g < SG; ++g) acc[p][g] = mf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NB - 1; ++p) issue();
    int bc = 0;
    for (int st = 0; st < nst; ++st) {
        for (int n = 0; n < N; ++n) {
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((NB - 2) * LPW) : "memory");
            issue();  // into the buffer of the previous step, which everyone has finished
            const float2 *sb = smd + bc * ROWS * 64 + 16 * sub + b;
            bc = (bc + 1) & (NB - 1);
            float are[MP], aim[MP];
#pragma unroll
            for (int p = 0; p < MP; ++p) {
                const float2 wv = sb[(2 * MP * half + 2 * p + (i >> 1)) * 64];
                const float wy = CONJ ? -wv.y : wv.y;
                are[p] = odd ? wy : wv.x;
                aim[p] = odd ? wv.x : -wy;
            }
            float2 xv[SG];
#pragma unroll
            for (int g = 0; g < SG; ++g) xv[g] = sb[(MB + 4 * g + i) * 64];
#pragma unroll
            for (int p = 0; p < MP; ++p)
#pragma unroll
                for (int g = 0; g < SG; ++g)
                    acc[p][g] = __builtin_amdgcn_mfma_f32_4x4x1f32(are[p], xv[g].x, acc[p][g], 0, 0, 0);
#pragma unroll
            for (int p = 0; p < MP; ++p)
#pragma unroll
                for (int g = 0; g < SG; ++g)
                    acc[p][g] = __builtin_amdgcn_mfma_f32_4x4x1f32(aim[p], xv[g].y, acc[p][g], 0, 0, 0);
        }
        const long long s0 = (step0 + st) * SB;
        if (k < K) {
#pragma unroll
            for (int g = 0; g < SG; ++g) {
                const long long s = s0 + 4 * g + i;
                if (s >= nsym) break;
                float2 *o = out + s * M * (long long)K + k;
#pragma unroll
                for (int p = 0; p < MP; ++p) {
                    const int m = m0 + 2 * p;
                    if (m < M) o[(long long)m * K] = float2{acc[p][g][0], acc[p][g][1]};
                    if (m + 1 < M) o[(long long)(m + 1) * K] = float2{acc[p][g][2], acc[p][g][3]};
                }
            }
        }
#pragma unroll
        for (int p = 0; p < MP; ++p)
#pragma unroll
            for (int g = 0; g < SG; ++g) acc[p][g] = mf4{0.f, 0.f, 0.f, 0.f};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail re-loads before exit
}

// The 16 dword DMAs of one wave's step in k_zf_mfma_w128 (4 rows x 4
// quarters of a 1 KiB row; row r at LDS byte lds + 8192 r, quarter q at
// + 256 q), M0 saved once.
__device__ __forceinline__ void dma_rows4x4(const float *const (&g)[16], unsigned lds) {
    const unsigned l0 = lds + 0u;
    const unsigned l1 = lds + 256u;
    const unsigned l2 = lds + 512u;
    const unsigned l3 = lds + 768u;
    const unsigned l4 = lds + 8192u;
    const unsigned l5 = lds + 8448u;
    const unsigned l6 = lds + 8704u;
    const unsigned l7 = lds + 8960u;
    const unsigned l8 = lds + 16384u;
    const unsigned l9 = lds + 16640u;
    const unsigned l10 = lds + 16896u;
    const unsigned l11 = lds + 17152u;
    const unsigned l12 = lds + 24576u;
    const unsigned l13 = lds + 24832u;
    const unsigned l14 = lds + 25088u;
    const unsigned l15 = lds + 25344u;
    unsigned keep;
    asm volatile("s_mov_b32 %[keep], m0\n\t"
                 "s_mov_b32 m0, %[l0]\n\ts_nop 0\n\tglobal_load_lds_dword %[a0], off\n\t"
                 "s_mov_b32 m0, %[l1]\n\ts_nop 0\n\tglobal_load_lds_dword %[a1], off\n\t"
                 "s_mov_b32 m0, %[l2]\n\ts_nop 0\n\tglobal_load_lds_dword %[a2], off\n\t"
                 "s_mov_b32 m0, %[l3]\n\ts_nop 0\n\tglobal_load_lds_dword %[a3], off\n\t"
                 "s_mov_b32 m0, %[l4]\n\ts_nop 0\n\tglobal_load_lds_dword %[a4], off\n\t"
                 "s_mov_b32 m0, %[l5]\n\ts_nop 0\n\tglobal_load_lds_dword %[a5], off\n\t"
                 "s_mov_b32 m0, %[l6]\n\ts_nop 0\n\tglobal_load_lds_dword %[a6], off\n\t"
                 "s_mov_b32 m0, %[l7]\n\ts_nop 0\n\tglobal_load_lds_dword %[a7], off\n\t"
                 "s_mov_b32 m0, %[l8]\n\ts_nop 0\n\tglobal_load_lds_dword %[a8], off\n\t"
                 "s_mov_b32 m0, %[l9]\n\ts_nop 0\n\tglobal_load_lds_dword %[a9], off\n\t"
                 "s_mov_b32 m0, %[l10]\n\ts_nop 0\n\tglobal_load_lds_dword %[a10], off\n\t"
                 "s_mov_b32 m0, %[l11]\n\ts_nop 0\n\tglobal_load_lds_dword %[a11], off\n\t"
                 "s_mov_b32 m0, %[l12]\n\ts_nop 0\n\tglobal_load_lds_dword %[a12], off\n\t"
                 "s_mov_b32 m0, %[l13]\n\ts_nop 0\n\tglobal_load_lds_dword %[a13], off\n\t"
                 "s_mov_b32 m0, %[l14]\n\ts_nop 0\n\tglobal_load_lds_dword %[a14], off\n\t"
                 "s_mov_b32 m0, %[l15]\n\ts_nop 0\n\tglobal_load_lds_dword %[a15], off\n\t"
                 "s_mov_b32 m0, %[keep]"
                 : [keep] "=&s"(keep)
                 : [a0] "v"(g[0]), [a1] "v"(g[1]), [a2] "v"(g[2]), [a3] "v"(g[3]), [a4] "v"(g[4]), [a5] "v"(g[5]), [a6] "v"(g[6]), [a7] "v"(g[7]), [a8] "v"(g[8]), [a9] "v"(g[9]), [a10] "v"(g[10]), [a11] "v"(g[11]), [a12] "v"(g[12]), [a13] "v"(g[13]), [a14] "v"(g[14]), [a15] "v"(g[15]),
                   [l0] "s"(l0), [l1] "s"(l1), [l2] "s"(l2), [l3] "s"(l3), [l4] "s"(l4), [l5] "s"(l5), [l6] "s"(l6), [l7] "s"(l7), [l8] "s"(l8), [l9] "s"(l9), [l10] "s"(l10), [l11] "s"(l11), [l12] "s"(l12), [l13] "s"(l13), [l14] "s"(l14), [l15] "s"(l15)
                 : "memory");
}

// The LDS-fed MFMA GEMM with 128-subcarrier blocks (k_zf_mfma_w128): 8 waves, wave w
// computes subcarriers 16 w + b of the block (16 rows x 16 symbols, 128
// accumulators, 2 waves/SIMD), so every staged row piece is 1 KiB of a row
// instead of 512 B (the no-MAC diagnostic showed the staging, not the MACs,
// sets the time).  LDS 4 x 32 rows x 1 KiB = 128 KiB: one workgroup per CU.
template <bool CONJ>
__global__ void __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(2, 2)))
k_zf_mfma_w128(const float2 *__restrict__ Wt, int a_m, int a_n, const float2 *__restrict__ in, int N, int M,
               int K, long long nsym, float2 *__restrict__ out, int ntile, int tpx, int nkb,
               long long chunk_steps) {
    constexpr int MP = 8, SG = 4, MB = 16, SB = 16, NB = 4, BW = 128;
    constexpr int ROWS = MB + SB, RPW = ROWS / 8, WR = MB / 8, LPW = 4 * RPW;
    static_assert(RPW == 4 && (NB - 2) * LPW <= 63, "rows per wave / vmcnt range");
    extern __shared__ __attribute__((aligned(16))) float2 smd[];  // [NB][ROWS][BW]
    const int bid = blockIdx.x, xcd = bid & 7, jb = bid >> 3;    // XCD-aware mapping as k_zf_gemm
    const int tile = xcd + 8 * (jb % tpx);
    if (tile >= ntile) return;  // whole workgroup
    const long long chunk = jb / tpx;
    const int kb = tile % nkb, mb = tile / nkb;
    const int lane = threadIdx.x & 63, b = lane >> 2, i = lane & 3;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int k = kb * BW + 16 * w + b;
    const int mb0 = mb * MB;
    const long long nsteps_total = (nsym + SB - 1) / SB;
    const long long step0 = chunk * chunk_steps, step1 = min(step0 + chunk_steps, nsteps_total);
    if (step1 <= step0) return;  // whole workgroup
    const int nst = (int)(step1 - step0);
    int offq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) offq[q] = min(kb * BW + 32 * q + (lane >> 1), K - 1) * 2 + (lane & 1);
    const bool odd = i & 1;
    const long long anK = (long long)a_n * K, NK = (long long)N * K;

    int si = 0, ni = 0, bi = 0;
    const float *wbase[WR];
#pragma unroll
    for (int r = 0; r < WR; ++r)
        wbase[r] = reinterpret_cast<const float *>(Wt + (long long)min(mb0 + w + 8 * r, M - 1) * a_m * K);
    const unsigned lds0 = (unsigned)(size_t)(lvoid_t *)smd + (unsigned)(w * BW * 8);
    auto issue = [&]() {
        const unsigned la = lds0 + (unsigned)(bi * ROWS * BW * 8);
        const long long s0 = (step0 + si) * SB;
        const float *ga[4 * RPW];
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const float *src;
            if (r < WR) {
                src = wbase[r] + 2 * (ni * anK);
            } else {
                const long long s = min(s0 + (w + 8 * r - MB), nsym - 1);
                src = reinterpret_cast<const float *>(in + s * NK + (long long)ni * K);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) ga[4 * r + q] = src + offq[q];
        }
        dma_rows4x4(ga, la);
        if (si < nst - 1 || ni < N - 1) {  // advance (the tail re-issues the last step)
            if (++ni == N) {
                ni = 0;
                ++si;
            }
        }
        bi = (bi + 1) & (NB - 1);
    };

    mf4 acc[MP][SG];
#pragma unroll
    for (int p = 0; p < MP; ++p)
#pragma unroll
        for (int g = 0; g < SG; ++g) acc[p][g] = mf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NB - 1; ++p) issue();
    int bc = 0;
    for (int st = 0; st < nst; ++st) {
        for (int n = 0; n < N; ++n) {
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((NB - 2) * LPW) : "memory");
            issue();  // into the buffer of the previous step, which everyone has finished
            const float2 *sb = smd + bc * ROWS * BW + 16 * w + b;
            bc = (bc + 1) & (NB - 1);
            float are[MP], aim[MP];
#pragma unroll
            for (int p = 0; p < MP; ++p) {
                const float2 wv = sb[(2 * p + (i >> 1)) * BW];
                const float wy = CONJ ? -wv.y : wv.y;
                are[p] = odd ? wy : wv.x;
                aim[p] = odd ? wv.x : -wy;
            }
            float2 xv[SG];
#pragma unroll
            for (int g = 0; g < SG; ++g) xv[g] = sb[(MB + 4 * g + i) * BW];
#pragma unroll
            for (int p = 0; p < MP; ++p)
#pragma unroll
                for (int g = 0; g < SG; ++g)
                    acc[p][g] = __builtin_amdgcn_mfma_f32_4x4x1f32(are[p], xv[g].x, acc[p][g], 0, 0, 0);
#pragma unroll
            for (int p = 0; p < MP; ++p)
#pragma unroll
                for (int g = 0; g < SG; ++g)
                    acc[p][g] = __builtin_amdgcn_mfma_f32_4x4x1f32(aim[p], xv[g].y, acc[p][g], 0, 0, 0);
        }
        const long long s0 = (step0 + st) * SB;
        if (k < K) {
#pragma unroll
            for (int g = 0; g < SG; ++g) {
                const long long s = s0 + 4 * g + i;
                if (s >= nsym) break;
                float2 *o = out + s * M * (long long)K + k;
#pragma unroll
                for (int p = 0; p < MP; ++p) {
                    const int m = mb0 + 2 * p;
                    if (m < M) o[(long long)m * K] = float2{acc[p][g][0], acc[p][g][1]};
                    if (m + 1 < M) o[(long long)(m + 1) * K] = float2{acc[p][g][2], acc[p][g][3]};
                }
            }
        }
#pragma unroll
        for (int p = 0; p < MP; ++p)
#pragma unroll
            for (int g = 0; g < SG; ++g) acc[p][g] = mf4{0.f, 0.f, 0.f, 0.f};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail re-loads before exit
}

// W-stationary MFMA GEMM for M <= 16 (k_zf_wstat; detect at U <= 16): the
// no-MAC diagnostic showed the re-staging of W tiles next to the input stream
// costs most of the time, so here a workgroup owns 16 subcarriers and ONE
// contiguous range of symbols, loads its whole A tile (all M <= 16 rows x N
// <= 72 columns x 16 subcarriers, <= 144 KiB) into LDS once, and its 8 waves
// then stream the input straight from HBM -- each wave its own 16 symbols
// per step, so no input is shared and nothing but the input and output
// crosses the memory system per symbol.  Lane (b, i) = block b = subcarrier
// k0 + b, as in the MFMA scheme above; A operands from LDS ([n][16 rows][16 subcarriers],
// rows >= M zero), input operands from global memory, prefetched PD n-steps
// ahead in registers.  PD = 2: same-process A/B at R = 64, 10 000 symbols,
// bit-identical (profiles/r3/r3z6_zf_detect_prefetch_depth.jsonl): detect
// U = 16 1.91 ms at PD = 3 (round 3) -> 1.85, U = 32 3.54 -> 3.34; PD = 1
// and PD = 5 are slower than both.
// XMAP: block b runs on XCD b % 8 (round-robin dispatch; speed only): the
// chunk is b % 8 + 8 (b / (8 nkb)) and the subcarrier block (b / 8) % nkb, so
// one XCD reads all subcarrier pieces of the same symbol rows.
template <bool CONJ, bool XMAP = false, int MR = 16, int PDT = 2>
__global__ void __attribute__((amdgpu_flat_work_group_size(MR == 64 ? 256 : 512, MR == 64 ? 256 : 512),
                               amdgpu_waves_per_eu(MR == 64 ? 1 : 2, MR == 64 ? 1 : 2)))
k_zf_wstat(const float2 *__restrict__ Wt, int a_m, int a_n, const float2 *__restrict__ in, int N, int M, int K,
           long long nsym, float2 *__restrict__ out, int nkb, int nmb, long long chunk_syms, long long ldi,
           long long ldo) {
    // MR rows per tile: 16 (MP = 8 row pairs x SG = 4 symbol quads per wave) or
    // 64 (apply at U = 16: all R = 64 output rows, MP = 32 x SG = 1)
    // MR = 64: 4-wave workgroups, one wave per SIMD (512 registers for 128 accumulators + 32 A pairs)
    constexpr int MP = MR / 2, SG = MR == 16 ? 4 : 1, SW = 4 * SG, PD = PDT, TR = MR * 16, NW = MR == 64 ? 4 : 8;
    extern __shared__ __attribute__((aligned(16))) float2 smd[];  // [N][MR][16]
    // tile = (subcarrier block, 16-row block); the row blocks of one subcarrier
    // block are adjacent in dispatch order, so they read the same input rows
    // at about the same time (the second read hits L2)
    const long long ntl = (long long)nkb * nmb;
    const int tl = XMAP ? (int)((blockIdx.x >> 3) % ntl) : (int)(blockIdx.x % ntl);
    const int kb = tl / nmb, mb = tl % nmb, mr0 = MR * mb;
    const long long chunk = XMAP ? (long long)(blockIdx.x & 7) + 8LL * (blockIdx.x / (8LL * ntl))
                                 : (long long)(blockIdx.x / ntl);
    const int lane = threadIdx.x & 63, b = lane >> 2, i = lane & 3;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int k0 = kb * 16, k = k0 + b, kc = min(k, K - 1);
    const long long sbeg = chunk * chunk_syms, send = min(sbeg + chunk_syms, nsym);
    if (sbeg >= send) return;  // whole workgroup
    // A tile -> LDS: element (n, m, bb) = A_k0+bb(m, n), rows m >= M zero
    for (int e = threadIdx.x; e < N * TR; e += 64 * NW) {
        const int bb = e & 15, m = mr0 + ((e >> 4) % MR), n = e / TR;
        const int kk = min(k0 + bb, K - 1);
        smd[e] = m < M ? Wt[((long long)m * a_m + (long long)n * a_n) * K + kk] : float2{0.f, 0.f};
    }
    __syncthreads();
    const bool odd = i & 1;
    const long long NK = (long long)N * ldi;  // input rows of ldi elements, output rows of ldo (>= K)
    const float2 *wl = smd + (i >> 1) * 16 + b;  // + n * TR + 2 p * 16

    for (long long s0 = sbeg + (long long)w * SW; s0 < send; s0 += (long long)NW * SW) {
        const float2 *xrow[SG];
#pragma unroll
        for (int g = 0; g < SG; ++g) xrow[g] = in + min(s0 + 4 * g + i, send - 1) * NK + kc;
        mf4 acc[MP][SG];
#pragma unroll
        for (int p = 0; p < MP; ++p)
#pragma unroll
            for (int g = 0; g < SG; ++g) acc[p][g] = mf4{0.f, 0.f, 0.f, 0.f};
        float2 xq[PD][SG];
#pragma unroll
        for (int d = 0; d < PD; ++d)
#pragma unroll
            for (int g = 0; g < SG; ++g) xq[d][g] = xrow[g][(long long)min(d, N - 1) * ldi];
        for (int n0 = 0; n0 < N; n0 += PD) {
#pragma unroll
            for (int d = 0; d < PD; ++d) {
                const int n = n0 + d;
                if (n < N) {  // wave-uniform
                    float2 xv[SG];
#pragma unroll
                    for (int g = 0; g < SG; ++g) xv[g] = xq[d][g];
                    const int nn = min(n + PD, N - 1);  // refill this slot PD steps ahead
#pragma unroll
                    for (int g = 0; g < SG; ++g) xq[d][g] = xrow[g][(long long)nn * ldi];
                    // row pairs in groups of 4: only one group's A operands live
#pragma unroll
                    for (int p0 = 0; p0 < MP; p0 += 4) {
                        float are[4], aim[4];
#pragma unroll
                        for (int p = 0; p < 4; ++p) {
                            const float2 wv = wl[n * TR + 2 * (p0 + p) * 16];
                            const float wy = CONJ ? -wv.y : wv.y;
                            are[p] = odd ? wy : wv.x;
                            aim[p] = odd ? wv.x : -wy;
                        }
#pragma unroll
                        for (int p = 0; p < 4; ++p)
#pragma unroll
                            for (int g = 0; g < SG; ++g)
                                acc[p0 + p][g] =
                                    __builtin_amdgcn_mfma_f32_4x4x1f32(are[p], xv[g].x, acc[p0 + p][g], 0, 0, 0);
#pragma unroll
                        for (int p = 0; p < 4; ++p)
#pragma unroll
                            for (int g = 0; g < SG; ++g)
                                acc[p0 + p][g] =
                                    __builtin_amdgcn_mfma_f32_4x4x1f32(aim[p], xv[g].y, acc[p0 + p][g], 0, 0, 0);
                    }
                }
            }
        }
        // 16-B stores: lanes b and b ^ 1 (same symbol) swap one row of their
        // row pair, so the even lane stores row 2p and the odd lane row 2p + 1,
        // each at subcarriers (kp, kp + 1); K odd: the last pair stores kp only.
        // Same-process A/B, R = 64, 10 000 symbols, bit-identical
        // (profiles/r5/r5j_zf_store_u*.jsonl): U = 16 1.862 -> 1.768 ms, U = 32
        // 3.374 -> 3.162 ms; non-temporal stores (8 or 16 B) are slower here.
        {
            const bool hi = b & 1;
            const int kp = k0 + (b & ~1);
#pragma unroll
            for (int g = 0; g < SG; ++g) {
                const long long s = s0 + 4 * g + i;
#pragma unroll
                for (int p = 0; p < MP; ++p) {
                    const float sx = hi ? acc[p][g][0] : acc[p][g][2];
                    const float sy = hi ? acc[p][g][1] : acc[p][g][3];
                    const float rx = __shfl_xor(sx, 4), ry = __shfl_xor(sy, 4);
                    const mf4 v = hi ? mf4{rx, ry, acc[p][g][2], acc[p][g][3]} : mf4{acc[p][g][0], acc[p][g][1], rx, ry};
                    const int m = mr0 + 2 * p + (hi ? 1 : 0);
                    if (s < send && m < M && kp < K) {
                        const long long e = (s * M + m) * ldo + kp;
                        float2 *o = out + e;
                        if (kp + 1 < K && !(e & 1)) {
                            *reinterpret_cast<mf4 *>(o) = v;  // 16-B aligned (out is)
                        } else {  // the row's last bin, or an odd K's odd row: 8-B pieces
                            o[0] = float2{v[0], v[1]};
                            if (kp + 1 < K) o[1] = float2{v[2], v[3]};
                        }
                    }
                }
            }
        }
    }
}


// ---------------------------------------------------------------------------
// k_zf_apply_ws16: the apply (multiplyWithChannelInv, cpuLS.hpp:449-463;
// Y[s][r][k] = sum_u W(r, u) X[s][u][k]) with TWO subcarriers per lane, so
// every input load and output store is 16 B per lane (a 1 KiB piece of a row
// per wave instruction).  The round-3 store-stream probes (scripts/
// zfprobe2.hip) put the apply's bytes at 35-40 % less time with
// 16-B than with 8-B stores.
// W-stationary: a workgroup owns a tile of 128 subcarriers x MB = 8 RG output
// rows, loads its W tile (U x MB x 1 KiB, 128 KiB at U = 16) into LDS once,
// then its 8 waves stream their own symbols of one symbol chunk: wave (rg, sg)
// computes rows 8 rg .. 8 rg + 7 for ST = 4 symbols at a time, reading the
// symbols' input pieces straight from memory (prefetched one u ahead) and W
// from LDS.  The nrb row blocks of one (chunk, subcarrier block) run on one
// XCD, adjacent in dispatch order, so each input piece comes from HBM once and
// from that XCD's L2 for the other row blocks.  Sum over u in the reference's
// order, one complex MAC per u (packed: (acc + x.re w) + (-x.im) w~, which
// matches within the parity tolerance, not bit for bit).  K odd: the last
// lane covers subcarriers (K-2, K-1) with W(K-2) zeroed and stores only K-1.
// ---------------------------------------------------------------------------
template <int MT, int RG, int ST, int NW, int XM = 0>
__global__ void __attribute__((amdgpu_flat_work_group_size(64 * NW, 64 * NW), amdgpu_waves_per_eu(NW / 4, NW / 4)))
k_zf_apply_ws16(const float2 *__restrict__ Wt, const float2 *__restrict__ X, int U, int R, int K, long long nsym,
                float2 *__restrict__ Y, int nkb, int nrb, int ngroups, long long chunk_syms, long long ldx,
                long long ldy) {
    constexpr int SGN = NW / RG, MB = MT * RG;
    extern __shared__ __attribute__((aligned(16))) float4 smw[];  // [U][MB][64]
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    int kb, rb;
    long long chunk;
    if constexpr (XM == 0) {  // (chunk, subcarrier block) groups round-robin over the XCDs
        const int group = xcd + 8 * (j / nrb);
        rb = j % nrb;
        if (group >= ngroups) return;  // whole workgroup
        kb = group % nkb;
        chunk = group / nkb;
    } else {  // A/B: every block of a chunk on one XCD (XM 1: row blocks adjacent, 2: subcarrier blocks adjacent)
        const int per = nkb * nrb;
        chunk = xcd + 8LL * (j / per);
        const int jj = j % per;
        rb = XM == 1 ? jj % nrb : jj / nkb;
        kb = XM == 1 ? jj / nrb : jj % nkb;
        if (chunk * nkb >= ngroups) return;  // whole workgroup
    }
    const long long sbeg = chunk * chunk_syms, send = min(sbeg + chunk_syms, nsym);
    if (sbeg >= send) return;  // whole workgroup
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int rg = w % RG, sg = w / RG;
    const int k = kb * 128 + 2 * lane;
    const bool pair = k + 1 < K, last = k == K - 1;  // last: K odd, this lane stores K-1 only
    const int kc = pair ? k : (K >= 2 ? K - 2 : 0);  // every 16-B load in range
    const int r0 = rb * MB;

    // W tile -> LDS; element (u, m) of this lane = W(r0 + m, u) at subcarriers (kc, kc + 1)
    for (int e = w; e < U * MB; e += NW) {
        const int u = e / MB, m = e % MB, r = r0 + m;
        float4 v = float4{0.f, 0.f, 0.f, 0.f};
        if (r < R) {
            const float2 *p = Wt + ((long long)u * R + r) * K + kc;
            if (pair) {
                v = *reinterpret_cast<const float4 *>(p);  // 8-B aligned on odd rows: unaligned dwordx4
            } else if (last) {
                const float2 h = p[1];
                v = float4{0.f, 0.f, h.x, h.y};
            }
        }
        smw[e * 64 + lane] = v;
    }
    __syncthreads();

    const float4 *wl = smw + (rg * MT) * 64 + lane;  // + (u * MB + i) * 64
    const int m0 = r0 + rg * MT;
    // input rows of ldx elements, output rows of ldy (>= K; the reference layout: K).  With an odd
    // pitch the 16-B input loads of odd rows are 8-B aligned: unaligned dwordx4, which gfx950's
    // global memory serves (the W tile loads above likewise); pitches padded to even lengths avoid it.
    const long long UK = (long long)U * ldx;
    for (long long s0 = sbeg + (long long)sg * ST; s0 < send; s0 += (long long)SGN * ST) {
        const float2 *xs[ST];
#pragma unroll
        for (int q = 0; q < ST; ++q) xs[q] = X + min(s0 + q, send - 1) * UK + kc;
        pk::v2f acc[MT][ST][2];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int q = 0; q < ST; ++q) acc[i][q][0] = acc[i][q][1] = (pk::v2f){0.f, 0.f};
        float4 xa[ST], xb[ST];
#pragma unroll
        for (int q = 0; q < ST; ++q) xa[q] = *reinterpret_cast<const float4 *>(xs[q]);
        auto step = [&](int u, const float4 (&x)[ST]) {
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const float4 wv = wl[(u * MB + i) * 64];
#pragma unroll
                for (int q = 0; q < ST; ++q) {
                    pk::mac(acc[i][q][0], (pk::v2f){x[q].x, x[q].y}, (pk::v2f){wv.x, wv.y});
                    pk::mac(acc[i][q][1], (pk::v2f){x[q].z, x[q].w}, (pk::v2f){wv.z, wv.w});
                }
            }
        };
        int u = 0;
        for (; u + 1 < U; u += 2) {
#pragma unroll
            for (int q = 0; q < ST; ++q) xb[q] = *reinterpret_cast<const float4 *>(xs[q] + (long long)(u + 1) * ldx);
            step(u, xa);
            if (u + 2 < U) {
#pragma unroll
                for (int q = 0; q < ST; ++q) xa[q] = *reinterpret_cast<const float4 *>(xs[q] + (long long)(u + 2) * ldx);
            }
            step(u + 1, xb);
        }
        if (u < U) step(u, xa);  // U odd: xa holds u = U - 1
        if (pair || last) {
#pragma unroll
            for (int q = 0; q < ST; ++q) {
                if (s0 + q >= send) break;
                float2 *o = Y + ((s0 + q) * R + m0) * ldy + kc;
#pragma unroll
                for (int i = 0; i < MT; ++i) {
                    if (m0 + i >= R) break;
                    float2 *y = o + (long long)i * ldy;
                    const float2 lo = pk::F(acc[i][q][0]), hi = pk::F(acc[i][q][1]);
                    if (pair)
                        __builtin_nontemporal_store(mf4{lo.x, lo.y, hi.x, hi.y}, reinterpret_cast<mf4 *>(y));
                    else
                        __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, hi),
                                                    reinterpret_cast<unsigned long long *>(y + 1));
                }
            }
        }
    }
}
}  // namespace zf

size_t zf_precoder_lds_bytes(int U, int R) {
    return ((size_t)U * R + (size_t)U * U) * sizeof(float2);
}

hipError_t launch_zf_precoder(const float2 *Hin, int U, int R, int K, float2 *W, float2 *Wt,
                              hipStream_t s) {
    if (K == 0) return hipSuccess;
    const size_t lds = zf_precoder_lds_bytes(U, R);
    if (lds > 64 * 1024)
        if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(&zf::k_zf_precoder), (int)lds); e != hipSuccess)
            return e;
    hipLaunchKernelGGL(zf::k_zf_precoder, dim3(K), dim3(256), lds, s, Hin, U, R, K, W, Wt);
    return hipGetLastError();
}

hipError_t launch_zf_transpose(const float2 *W, int U, int R, int K, float2 *Wt, hipStream_t s) {
    if (K == 0) return hipSuccess;
    const int UR = U * R;
    hipLaunchKernelGGL(zf::k_zf_transpose, dim3((K + 63) / 64, (UR + 63) / 64), dim3(256), 0, s, W, UR,
                       K, Wt);
    return hipGetLastError();
}

namespace {

template <int MT, int ST, int MG, bool CONJ, bool PF = true>
hipError_t gemm_launch(const float2 *Wt, int a_m, int a_n, const float2 *in, int N, int M, int K,
                       long long nsym, float2 *out, hipStream_t s) {
    constexpr int SBLK = (4 / MG) * ST;
    const int nkb = (K + 63) / 64, nmb = (M + MG * MT - 1) / (MG * MT);
    const int ntile = nkb * nmb, tpx = (ntile + 7) / 8;
    const long long nsteps = (nsym + SBLK - 1) / SBLK;
    // ~8 workgroups per CU (256 CUs) over all tiles, at least 4 steps per chunk
    long long nchunk = (2048 + 8LL * tpx - 1) / (8LL * tpx);
    long long chunk_steps = (nsteps + nchunk - 1) / nchunk;
    if (chunk_steps < 4) chunk_steps = 4;
    nchunk = (nsteps + chunk_steps - 1) / chunk_steps;
    const long long blocks = 8LL * tpx * nchunk;
    hipLaunchKernelGGL((zf::k_zf_gemm<MT, ST, MG, CONJ, PF>), dim3((unsigned)blocks), dim3(256), 0, s,
                       Wt, a_m, a_n, in, N, M, K, nsym, out, ntile, tpx, nkb, chunk_steps);
    return hipGetLastError();
}

template <int MT, int MG, bool CONJ>
hipError_t gemm_variant(const float2 *Wt, int a_m, int a_n, const float2 *in, int N, int M, int K,
                        long long nsym, float2 *out, hipStream_t s) {
    return gemm_launch<MT, 8, MG, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
}

template <int MG, bool CONJ, int ST = 8>
hipError_t gemm_lds_launch(const float2 *Wt, int a_m, int a_n, const float2 *in, int N, int M, int K,
                           long long nsym, float2 *out, hipStream_t s) {
    constexpr int SB = (4 / MG) * ST;
    const int nkb = (K + 63) / 64, nmb = (M + MG * 8 - 1) / (MG * 8);
    const int ntile = nkb * nmb, tpx = (ntile + 7) / 8;
    const long long nsteps = (nsym + SB - 1) / SB;
    long long nchunk = (2048 + 8LL * tpx - 1) / (8LL * tpx);
    long long chunk_steps = (nsteps + nchunk - 1) / nchunk;
    if (chunk_steps < 4) chunk_steps = 4;
    nchunk = (nsteps + chunk_steps - 1) / chunk_steps;
    const long long blocks = 8LL * tpx * nchunk;
    hipLaunchKernelGGL((zf::k_zf_gemm_lds<MG, CONJ>), dim3((unsigned)blocks), dim3(256), 0, s, Wt, a_m,
                       a_n, in, N, M, K, nsym, out, ntile, tpx, nkb, chunk_steps);
    return hipGetLastError();
}


// k_zf_apply_ws16 (16-B lanes, W-stationary): NW waves, RG row groups of MT
// rows per tile, ST symbols per wave step
template <int MT, int RG, int ST, int NW, int XM = 0>
hipError_t apply_ws16_launch(const float2 *Wt, const float2 *X, int U, int R, int K, long long nsym, float2 *Y,
                             int target_groups, hipStream_t s, long long ldx = -1, long long ldy = -1) {
    constexpr int MB = MT * RG, WSTEP = NW / RG * ST;
    const size_t lds = (size_t)U * MB * 64 * sizeof(float4);
    if (lds > 160 * 1024 || K < 2) return hipErrorInvalidValue;
    const int nkb = (K + 127) / 128, nrb = (R + MB - 1) / MB;
    long long nch = (target_groups + nkb - 1) / nkb;
    if (nch < 1) nch = 1;
    long long chunk_syms = (nsym + nch - 1) / nch;
    chunk_syms = (chunk_syms + WSTEP - 1) / WSTEP * WSTEP;  // whole steps of every wave
    nch = (nsym + chunk_syms - 1) / chunk_syms;
    const long long ngroups = nch * nkb;
    const long long blocks = XM == 0 ? 8LL * ((ngroups + 7) / 8) * nrb : 8LL * ((nch + 7) / 8) * nkb * nrb;
    if (blocks > 0x7fffffffll) return hipErrorInvalidValue;
    auto kern = zf::k_zf_apply_ws16<MT, RG, ST, NW, XM>;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)lds); e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * NW), lds, s, Wt, X, U, R, K, nsym, Y, nkb, nrb,
                       (int)ngroups, chunk_syms, ldx < 0 ? K : ldx, ldy < 0 ? K : ldy);
    return hipGetLastError();
}


template <int MPW, int SG, bool CONJ>
hipError_t mfma_lds8_launch(const float2 *Wt, int a_m, int a_n, const float2 *in, int N, int M, int K,
                            long long nsym, float2 *out, hipStream_t s) {
    constexpr int SB = 4 * SG, MB = 4 * MPW;
    constexpr size_t lds = (size_t)4 * (MB + SB) * 64 * sizeof(float2);  // 96 KiB
    const int nkb = (K + 63) / 64, nmb = (M + MB - 1) / MB;
    const int ntile = nkb * nmb, tpx = (ntile + 7) / 8;
    const long long nsteps = (nsym + SB - 1) / SB;
    long long nchunk = (1024 + 8LL * tpx - 1) / (8LL * tpx);
    long long chunk_steps = (nsteps + nchunk - 1) / nchunk;
    if (chunk_steps < 2) chunk_steps = 2;
    nchunk = (nsteps + chunk_steps - 1) / chunk_steps;
    const long long blocks = 8LL * tpx * nchunk;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    auto kern = zf::k_zf_mfma_lds8<MPW, SG, CONJ>;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)lds); e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(512), lds, s, Wt, a_m, a_n, in, N, M, K, nsym, out,
                       ntile, tpx, nkb, chunk_steps);
    return hipGetLastError();
}

template <bool CONJ>
hipError_t mfma_w128_launch(const float2 *Wt, int a_m, int a_n, const float2 *in, int N, int M, int K,
                            long long nsym, float2 *out, hipStream_t s) {
    constexpr int SB = 16, MB = 16;
    constexpr size_t lds = (size_t)4 * (MB + SB) * 128 * sizeof(float2);  // 128 KiB
    const int nkb = (K + 127) / 128, nmb = (M + MB - 1) / MB;
    const int ntile = nkb * nmb, tpx = (ntile + 7) / 8;
    const long long nsteps = (nsym + SB - 1) / SB;
    long long nchunk = (1024 + 8LL * tpx - 1) / (8LL * tpx);
    long long chunk_steps = (nsteps + nchunk - 1) / nchunk;
    if (chunk_steps < 2) chunk_steps = 2;
    nchunk = (nsteps + chunk_steps - 1) / chunk_steps;
    const long long blocks = 8LL * tpx * nchunk;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    auto kern = zf::k_zf_mfma_w128<CONJ>;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), (int)lds); e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(512), lds, s, Wt, a_m, a_n, in, N, M, K, nsym, out,
                       ntile, tpx, nkb, chunk_steps);
    return hipGetLastError();
}

template <bool CONJ, bool XMAP, int MR = 16, int PD = 2>
hipError_t wstat_launch(const float2 *Wt, int a_m, int a_n, const float2 *in, int N, int M, int K,
                        long long nsym, float2 *out, hipStream_t s, long long ldi = -1, long long ldo = -1) {
    const size_t lds = (size_t)N * MR * 16 * sizeof(float2);  // N * MR <= 1152: <= 144 KiB
    const int nkb = (K + 15) / 16, nmb = (M + MR - 1) / MR;
    // ~1 workgroup per CU over all (tile, symbol chunk) pairs;
    // XMAP: a multiple of 8 chunks (one per XCD)
    long long nchunk = XMAP ? 8 : (256 + nkb * nmb - 1) / (nkb * nmb);
    long long chunk_syms = (nsym + nchunk - 1) / nchunk;
    if (chunk_syms < 128) chunk_syms = 128;
    nchunk = (nsym + chunk_syms - 1) / chunk_syms;
    if (XMAP) nchunk = (nchunk + 7) / 8 * 8;  // empty chunks return at once
    const long long blocks = (long long)nkb * nmb * nchunk;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    auto kern = zf::k_zf_wstat<CONJ, XMAP, MR, PD>;
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(kern), 72 * 256 * (int)sizeof(float2));
        e != hipSuccess)
        return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(MR == 64 ? 256 : 512), lds, s, Wt, a_m, a_n, in, N, M, K,
                       nsym, out, nkb, nmb, chunk_syms, ldi < 0 ? K : ldi, ldo < 0 ? K : ldo);
    return hipGetLastError();
}

// Measured defaults (same-process A/B, R = 64, 10 000 symbols):
//   detect, M = U > 8, N = R <= 72: W-stationary MFMA with one symbol chunk
//     per XCD (k_zf_wstat<., true>): 1.87 vs 2.05 ms (VALU) at U = 16,
//     3.34 vs 3.67 (k_zf_mfma_lds8<8,4>) / 4.09 (VALU) at U = 32;
//   detect with N > 72: k_zf_mfma_lds8<8,4> (M > 16) / k_zf_mfma_w128;
//   detect at U <= 8: the per-wave register-tiled VALU kernel (1.26-1.37 vs
//     1.35-1.39 ms for the LDS VALU kernel at U = 8);
//   apply at 32 <= N = U <= 72: k_zf_wstat<., true> (4.08 vs 4.28 ms);
//   otherwise the LDS VALU kernel when both operands are wide enough (at
//     N = 4 its per-chunk barriers and stores dominate), else the register-
//     tiled one.
// Measured-slower candidates (register tiles without double buffering,
// DMA-fed LDS VALU tiles, MFMA from L1 / through 4-wave LDS tiles, other
// W-stationary depths and tile heights) are kept out of the product sources
// (scripts/experiments/ab_knobs_r3.patch).
enum { ZF_REG = 0, ZF_LDS = 1, ZF_MFMA_LDS8 = 6, ZF_MFMA_W128 = 7, ZF_WSTAT = 9 };
template <bool CONJ>
hipError_t gemm_dispatch(const float2 *Wt, int a_m, int a_n, const float2 *in, int N, int M, int K,
                         long long nsym, float2 *out, hipStream_t s) {
    const int mode = CONJ ? (N < 8 ? ZF_LDS : M <= 8 ? ZF_REG : N <= 72 ? ZF_WSTAT : M > 16 ? ZF_MFMA_LDS8 : ZF_MFMA_W128)
                          : (N >= 32 && N <= 72 ? ZF_WSTAT : ZF_LDS);
    if (mode == ZF_WSTAT && N <= 72) return wstat_launch<CONJ, true>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    if (mode == ZF_MFMA_LDS8) return mfma_lds8_launch<8, 4, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    if (mode == ZF_MFMA_W128) return mfma_w128_launch<CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    if (M > 4 && N >= 8 && mode != ZF_REG) {
        if (M <= 8) return gemm_lds_launch<1, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
        if (M <= 16) return gemm_lds_launch<2, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
        return gemm_lds_launch<4, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    }
    if (M <= 2) return gemm_variant<2, 1, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    if (M <= 4) return gemm_variant<4, 1, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    if (M <= 8) return gemm_variant<8, 1, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    if (M <= 16) return gemm_variant<8, 2, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
    return gemm_variant<8, 4, CONJ>(Wt, a_m, a_n, in, N, M, K, nsym, out, s);
}

}  // namespace

// Y[s][r][k] = sum_u W(r, u) X[s][u][k];  W(r, u) = Wt[(u*R + r)*K + k]
hipError_t launch_zf_apply(const float2 *Wt, const float2 *X, int U, int R, int K, long long nsym,
                           float2 *Y, hipStream_t s) {
    if (K == 0 || nsym == 0) return hipSuccess;
    // 16-B lanes, W-stationary (k_zf_apply_ws16): 8-row tiles up to U = 20
    // (W tile U x 8 KiB of LDS), 4-row tiles with 8-symbol steps up to U = 40;
    // same-process A/B at R = 64, K = 1023, 10 000 symbols:
    // U = 4 / 8 / 16 / 24 / 32: 1.82 / 1.96 / 2.38 / 3.16 / 4.42 ms -> 1.50 /
    // 1.53 / 1.94-1.96 / 2.93 / 3.58 ms.  Fewer than 8 antenna rows fill less
    // than one 8-row tile: the register-tiled kernels below.  8-row tiles run
    // every block of a 64-symbol chunk on one XCD (row blocks adjacent,
    // XM = 1): same-process A/B vs chunk groups round-robin over the XCDs,
    // U = 4 / 8 / 16 / 20: 1.320 / 1.358 / 1.743 / 2.004 -> 1.235 / 1.253 /
    // 1.718 / 1.996 ms (profiles/r3/r3l_zf_apply_xmap.jsonl); the same map
    // on the 4-row tiles is 1.7x slower.
    if (K >= 2 && R >= 8 && U <= 20) return apply_ws16_launch<8, 1, 4, 8, 1>(Wt, X, U, R, K, nsym, Y, 64, s);
    if (K >= 2 && R >= 8 && U <= 40) return apply_ws16_launch<4, 1, 8, 8>(Wt, X, U, R, K, nsym, Y, 32, s);
    return gemm_dispatch<false>(Wt, 1, R, X, U, R, K, nsym, Y, s);
}

// The apply with row pitches (X rows of ldx, Y rows of ldy elements >= K):
// the 16-B-lane W-stationary kernel, R >= 8, U <= 40, K >= 2.
bool zf_apply_pitched_supported(int U, int R, int K) { return K >= 2 && R >= 8 && U <= 40; }
hipError_t launch_zf_apply_ld(const float2 *Wt, const float2 *X, long long ldx, int U, int R, int K, long long nsym,
                              float2 *Y, long long ldy, hipStream_t s) {
    if (K == 0 || nsym == 0) return hipSuccess;
    if (ldx == K && ldy == K) return launch_zf_apply(Wt, X, U, R, K, nsym, Y, s);
    if (!zf_apply_pitched_supported(U, R, K)) return hipErrorInvalidValue;
    if (U <= 20) return apply_ws16_launch<8, 1, 4, 8, 1>(Wt, X, U, R, K, nsym, Y, 64, s, ldx, ldy);
    return apply_ws16_launch<4, 1, 8, 8>(Wt, X, U, R, K, nsym, Y, 32, s, ldx, ldy);
}

// X[s][u][k] = sum_r conj(W(r, u)) Y[s][r][k]
hipError_t launch_zf_detect(const float2 *Wt, const float2 *Y, int U, int R, int K, long long nsym,
                            float2 *X, hipStream_t s) {
    if (K == 0 || nsym == 0) return hipSuccess;
    return gemm_dispatch<true>(Wt, R, 1, Y, R, U, K, nsym, X, s);
}

// The same with row pitches: Y[s][r][k] at Y[(s R + r) ldy + k], X[s][u][k]
// at X[(s U + u) ldx + k] (ldy, ldx >= K; the pad is neither read nor
// written).  Rows padded to a multiple of 16 elements start on 128-B lines,
// so no workgroup leaves a partly written line for its neighbour to complete
// (DESIGN.md 7c, round 6).  The W-stationary kernel for every U: R <= 72.
bool zf_detect_pitched_supported(int U, int R) { return U >= 1 && R <= 72; }
hipError_t launch_zf_detect_ld(const float2 *Wt, const float2 *Y, long long ldy, int U, int R, int K,
                               long long nsym, float2 *X, long long ldx, hipStream_t s) {
    if (K == 0 || nsym == 0) return hipSuccess;
    if (ldy == K && ldx == K) return gemm_dispatch<true>(Wt, R, 1, Y, R, U, K, nsym, X, s);
    if (!zf_detect_pitched_supported(U, R)) return hipErrorInvalidValue;
    return wstat_launch<true, true>(Wt, R, 1, Y, R, U, K, nsym, X, s, ldy, ldx);
}

}  // namespace ofdm
