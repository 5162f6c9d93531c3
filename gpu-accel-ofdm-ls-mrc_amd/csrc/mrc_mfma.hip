// mrc_mfma.hip -- the antenna combine as a matrix-core (MFMA) product, for
// the comparison BASELINE.json configs[4] asks for ("compare MFMA-cgemm vs
// elementwise combine").  Same contract as k_mrc_freq<BIN_LAYOUT> (bin-layout
// Hc [F][R][C], bin-indexed P [F][C], frequency-domain data symbols).
//
// Per subcarrier b the combine is a complex matrix-VECTOR product,
//   N[s][b] = sum_r Y[s][r][b] Hc[r][b]       (matrixMultThenSum, cpuLS.hpp:187-208)
// so there is no shared right-hand side across subcarriers to fill a GEMM
// tile.  The densest MFMA form: v_mfma_f32_16x16x4f32 per subcarrier with
//   A[s][k] = Y[s][r0 + k/2][b].(re, im)[k%2]     16 symbols x 2 antennas
//   B[k][0] = (Hr, -Hi)[k%2],  B[k][1] = (Hi, Hr)[k%2],  B[k][n>1] = 0
//   D[s][0] = Re N, D[s][1] = Im N
// i.e. 2 of the 16 output columns are useful (12.5 % of the MFMA's flops).
// A wave owns 16 symbols x 16 bins and runs 16 MFMAs per antenna pair; the
// Y tile (32 rows x 128 B) is loaded coalesced (8 lanes per row) and turned
// into A operands through a conflict-free LDS image (pitch 34 floats).
#include "common.hpp"
#include "launch.hpp"

namespace ofdm {
namespace mfma {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int BINS = 16;     // bins per wave
constexpr int SYMS = 16;     // symbols per wave (= MFMA M)
constexpr int WAVES = 4;     // waves per workgroup: 64 consecutive bins
constexpr int PITCH = 34;    // floats per staged row (16 bins x 2 + 2 pad)
constexpr int ROWS = 32;     // 16 symbols x 2 antennas
constexpr int WLDS = ROWS * PITCH;

__global__ void __launch_bounds__(256) k_mrc_freq_mfma(
    const float2 *__restrict__ Y, long long frame_stride, long long sym_stride, long long nframes,
    int nsym, int R, int C, const float2 *__restrict__ Hc, long long hc_fstride,
    const float *__restrict__ P, long long p_fstride, float2 *__restrict__ out, int mode) {
    __shared__ __attribute__((aligned(16))) float lds[WAVES * WLDS];
    const int K = C - 1;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    float *img = lds + w * WLDS;
    const int bblocks = C / (BINS * WAVES);
    const int tiles = (nsym + SYMS - 1) / SYMS;
    const long long blk = blockIdx.x;
    const int bb = (int)(blk % bblocks);
    const long long ft = blk / bblocks;
    const long long f = ft / tiles;
    const int s0 = (int)(ft % tiles) * SYMS;
    if (f >= nframes) return;
    const int b0 = (bb * WAVES + w) * BINS;
    const float2 *Yf = Y + f * frame_stride;
    const float2 *Hf = Hc + f * hc_fstride;

    // coalesced load role: 8 lanes per row, 16 B each; rows ld = l / 8 + 8 i
    const int lr = l >> 3, lc = l & 7;
    // MFMA role: A row (symbol) i = l % 16, k = l / 16 = (antenna rr, component p)
    const int ai = l & 15, ak = l >> 4, arr = ak >> 1, ap = ak & 1;
    const int bn = l & 15;  // B column: 0 = re, 1 = im, others 0
    f4 acc[BINS];
#pragma unroll
    for (int j = 0; j < BINS; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};

    for (int r0 = 0; r0 < R; r0 += 2) {
        // stage Y rows (s0 + srow, r0 + rr) bins [b0, b0 + 16); row index = rr * 16 + srow
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = lr + 8 * i;
            const int rr = row >> 4, srow = row & 15;
            float4 v = float4{0.f, 0.f, 0.f, 0.f};
            if (s0 + srow < nsym && r0 + rr < R)
                v = *reinterpret_cast<const float4 *>(Yf + (long long)(s0 + srow) * sym_stride +
                                                      (long long)(r0 + rr) * C + b0 + 2 * lc);
            float *d = img + row * PITCH + 4 * lc;
            *reinterpret_cast<float2 *>(d) = float2{v.x, v.y};
            *reinterpret_cast<float2 *>(d + 2) = float2{v.z, v.w};
        }
        // B operands: Hc[r0 + arr][b0 + j] for the two useful columns
        float bv[BINS];
        if (bn < 2 && r0 + arr < R) {
            const float2 *hr = Hf + (long long)(r0 + arr) * C + b0;
#pragma unroll
            for (int j = 0; j < BINS; ++j) {
                const float2 h = hr[j];
                bv[j] = bn == 0 ? (ap == 0 ? h.x : -h.y) : (ap == 0 ? h.y : h.x);
            }
        } else {
#pragma unroll
            for (int j = 0; j < BINS; ++j) bv[j] = 0.f;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float *arow = img + (arr * 16 + ai) * PITCH + ap;
#pragma unroll
        for (int j = 0; j < BINS; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(arow[2 * j], bv[j], acc[j], 0, 0, 0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // D[s = 4 (l / 16) + v][n = l % 16]: lanes n = 0 / 1 hold Re / Im of 4 symbols.
    // Stage [16 symbols][16 bins] complex in the image, then store rows.
    if (bn < 2) {
#pragma unroll
        for (int j = 0; j < BINS; ++j)
#pragma unroll
            for (int v = 0; v < 4; ++v) img[(4 * (l >> 4) + v) * PITCH + 2 * j + bn] = acc[j][v];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // lane -> (symbol l / 4, bins 4 (l % 4) .. + 4)
    const int os = l >> 2, oj = 4 * (l & 3);
    if (s0 + os >= nsym) return;
    const long long q = f * nsym + s0 + os;
    float2 *o = out + q * K;
    const float *Pf = P + f * p_fstride;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int b = b0 + oj + j;
        if (b == 0) continue;  // DC bin dropped (cpuLS.hpp:290-292)
        float2 v = *reinterpret_cast<const float2 *>(img + os * PITCH + 2 * (oj + j));
        if (mode == 0) {
            const float p = Pf[b];
            o[out_pos(b - 1, K)] = float2{v.x * __builtin_amdgcn_rcpf(p), v.y * __builtin_amdgcn_rcpf(p)};
        } else {
            o[b - 1] = v;
        }
    }
}

}  // namespace mfma

hipError_t launch_mrc_freq_mfma(const float2 *Y, long long frame_stride, long long sym_stride,
                                long long nframes, int nsym, int R, int C, const float2 *Hc,
                                long long hc_fstride, const float *P, long long p_fstride,
                                float2 *out, int mode, hipStream_t s) {
    using namespace mfma;
    if (nframes <= 0 || nsym <= 0) return hipSuccess;
    if (C < BINS * WAVES) return hipErrorInvalidValue;
    const long long tiles = (nsym + SYMS - 1) / SYMS;
    const long long blocks = nframes * tiles * (C / (BINS * WAVES));
    if (blocks > 0x7fffffffll) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_mrc_freq_mfma, dim3((unsigned)blocks), dim3(64 * WAVES), 0, s, Y,
                       frame_stride, sym_stride, nframes, nsym, R, C, Hc, hc_fstride, P, p_fstride,
                       out, mode);
    return hipGetLastError();
}

}  // namespace ofdm
