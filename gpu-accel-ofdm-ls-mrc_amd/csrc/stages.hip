// stages.hip -- the reference's stage-wise GPU operations, for callers of the
// gpuLS per-stage API (gpuLS.cu:261-293).  The fused kernels (frame_td.hip,
// lsmrc_freq.hip) never materialise these intermediates; these exist so the
// individual methods keep their meaning:
//   k_conj_product   multiplyWithChannelConj (gpuLS.cu:212-233):
//                    prod[s][r][j] = Y[s][r][j+1] * Hconj[r][j]
//   k_combine        combineForMRC (gpuLS.cu:236-259) [+ shiftOneRow]:
//                    out[s][k] = sum_r prod[s][r][j] / Hsqrd[j], antennas in
//                    order (the reference's shared-memory tree also lacked a
//                    barrier, gpuLS.cu:245-247)
//   k_shift_rows     shiftOneRow (gpuLS.cu:109-125), out of place
//   k_dist_sqrd      findDistSqrd (gpuLS.cu:185-209, cpuLS.hpp:211-228) on an
//                    arbitrary R x K matrix, rows summed in order
//   k_export_estimate one frame's LS estimate from a frame workspace (the
//                    fused kernels' lane-ordered Hc rows, or the bin layout of
//                    the staged path) into the reference's layout: Hconj
//                    [R][K], Hsqrd [K] -- what demodOneFrameCUDA leaves in its
//                    Hconj / Hsqrd arguments (gpuLS.cu:617-629)
#include "common.hpp"
#include "launch.hpp"

namespace ofdm {

__global__ void __launch_bounds__(256) k_conj_product(const float2 *__restrict__ Y, long long rows,
                                                      int R, int C, const float2 *__restrict__ Hc,
                                                      float2 *__restrict__ prod) {
    const int K = C - 1;
    const long long row = blockIdx.y;  // s * R + r
    const int r = (int)(row % R);
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < K; j += gridDim.x * blockDim.x)
        prod[row * K + j] = cmul(Y[row * C + j + 1], Hc[(long long)r * K + j]);
}

__global__ void __launch_bounds__(256) k_combine(const float2 *__restrict__ prod, int R, int K,
                                                 const float *__restrict__ P, int rotate,
                                                 float2 *__restrict__ out) {
    const long long s = blockIdx.y;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < K; j += gridDim.x * blockDim.x) {
        float2 acc = prod[s * R * K + j];
        for (int r = 1; r < R; ++r) acc = cadd(acc, prod[(s * R + r) * K + j]);
        const float p = P[j];
        out[s * K + (rotate ? out_pos_any(j, K) : j)] = float2{acc.x / p, acc.y / p};
    }
}

__global__ void __launch_bounds__(256) k_shift_rows(const float2 *__restrict__ in, int K,
                                                    float2 *__restrict__ out) {
    const long long row = blockIdx.y;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < K; j += gridDim.x * blockDim.x)
        out[row * K + out_pos_any(j, K)] = in[row * K + j];
}

__global__ void __launch_bounds__(256) k_dist_sqrd(const float2 *__restrict__ H, int R, int K,
                                                   float *__restrict__ P) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    float p = 0.f;
    for (int r = 0; r < R; ++r) {
        const float2 h = H[(long long)r * K + j];
        p = (r == 0) ? (h.x * h.x) + (h.y * h.y) : p + (h.x * h.x) + (h.y * h.y);
    }
    P[j] = p;
}

// Position of bin b (1 <= b < C) inside one lane-ordered Hc row of C float2
// (frame_td.hip / frame_td2048.hip / frame_td4096.hip: lane t of a wave owns
// the bins b0(t) + 16 k, b0(t) = (t >> 2) + 256 c(t & 3), c(a) = (a >> 1) + 2 (a & 1)).
// Other C: bin layout (position = b).
__device__ __forceinline__ int lane_of(int b, int &k) {  // b < 1024
    const int q = b & 15, c = b >> 8;
    k = (b >> 4) & 15;
    return 4 * q + (((c & 1) << 1) | (c >> 1));
}
__device__ __forceinline__ int hc_pos(int b, int C) {  // C = 0: bin layout
    int k;
    if (C == 1024) {  // float4 (k >> 1) * 64 + t holds bins (k & ~1, k | 1) of lane t
        const int t = lane_of(b, k);
        return 2 * ((k >> 1) * 64 + t) + (k & 1);
    }
    if (C == 2048) {  // float4 k * 64 + t = (Hc[2 b'], Hc[2 b' + 1]), b' = b0(t) + 16 k
        const int t = lane_of(b >> 1, k);
        return 2 * (k * 64 + t) + (b & 1);
    }
    if (C == 1536) {  // frame_td_fft512.hip: slot 8 j + d of lane 8 s + c holds bin 3 (s + 8 c + 64 d) + j
        const int q = b / 3, j = b - 3 * q;
        return (8 * j + (q >> 6)) * 64 + 8 * (q & 7) + ((q >> 3) & 7);
    }
    if (C == 3072) {  // wave e, slot 8 j + d of lane 8 s + c holds bin 3 (2 (s + 8 c + 64 d) + e) + j
        const int q = b / 3, j = b - 3 * q, e = q & 1, kk = q >> 1;
        return e * 1536 + (8 * j + (kk >> 6)) * 64 + 8 * (kk & 7) + ((kk >> 3) & 7);
    }
    if (C == 512 || C == 256 || C == 128) {  // P = C / 64: slot d of lane 8 s + c holds bin s + P c + 8 P d
        const int np = C >> 6, lw = 8 * np;
        return (b / lw) * lw + 8 * (b % np) + ((b / np) & 7);
    }
    if (C == 6144) {  // wave e, slot 8 j + d of lane 8 s + c holds bin 3 (4 (s + 8 c + 64 d) + e) + j
        const int q = b / 3, j = b - 3 * q, e = q & 3, kk = q >> 2;
        return e * 1536 + (8 * j + (kk >> 6)) * 64 + 8 * (kk & 7) + ((kk >> 3) & 7);
    }
    if (C == 4096) {  // float2 e * 2048 + h * 1024 + (k >> 1) * 128 + 2 t + (k & 1) = Hc[4 b' + 2 h + e]
        const int t = lane_of(b >> 2, k);
        return (b & 1) * 2048 + ((b >> 1) & 1) * 1024 + (k >> 1) * 128 + 2 * t + (k & 1);
    }
    return b;
}

__global__ void __launch_bounds__(256) k_export_estimate(const float2 *__restrict__ Hc,
                                                         const float *__restrict__ P, int R, int C,
                                                         int lay, float2 *__restrict__ Hconj,
                                                         float *__restrict__ Hsqrd) {
    const int K = C - 1;
    const int r = blockIdx.y;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < K; j += gridDim.x * blockDim.x) {
        Hconj[(long long)r * K + j] = Hc[(long long)r * C + hc_pos(j + 1, lay)];
        if (r == 0 && Hsqrd) Hsqrd[j] = P[j + 1];
    }
}

hipError_t launch_export_estimate(const float2 *Hc, const float *P, int R, int C, bool lane_order,
                                  float2 *Hconj, float *Hsqrd, hipStream_t s) {
    if (R > 65535) return hipErrorInvalidValue;
    const int lay = lane_order ? C : 0;
    hipLaunchKernelGGL(k_export_estimate, dim3((unsigned)((C - 1 + 255) / 256), (unsigned)R), dim3(256), 0, s,
                       Hc, P, R, C, lay, Hconj, Hsqrd);
    return hipGetLastError();
}

static dim3 grid_rows(int K, long long rows) {
    return dim3((unsigned)((K + 255) / 256), (unsigned)rows);
}

hipError_t launch_conj_product(const float2 *Y, long long nsyms, int R, int C, const float2 *Hc,
                               float2 *prod, hipStream_t s) {
    const long long rows = nsyms * R;
    // chunks start on symbol boundaries so that r = row % R holds per chunk
    const long long chunk = (65535 / R) * R;
    if (chunk == 0) return hipErrorInvalidValue;
    for (long long r0 = 0; r0 < rows; r0 += chunk) {
        const long long n = rows - r0 < chunk ? rows - r0 : chunk;
        hipLaunchKernelGGL(k_conj_product, grid_rows(C - 1, n), dim3(256), 0, s, Y + r0 * C, n, R, C,
                           Hc, prod + r0 * (C - 1));
    }
    return hipGetLastError();
}

hipError_t launch_combine(const float2 *prod, long long nsyms, int R, int K, const float *P,
                          int rotate, float2 *out, hipStream_t s) {
    for (long long s0 = 0; s0 < nsyms; s0 += 65535) {
        const long long n = nsyms - s0 < 65535 ? nsyms - s0 : 65535;
        hipLaunchKernelGGL(k_combine, grid_rows(K, n), dim3(256), 0, s, prod + s0 * R * K, R, K, P,
                           rotate, out + s0 * K);
    }
    return hipGetLastError();
}

hipError_t launch_shift_rows(const float2 *in, long long nrows, int K, float2 *out, hipStream_t s) {
    for (long long r0 = 0; r0 < nrows; r0 += 65535) {
        const long long n = nrows - r0 < 65535 ? nrows - r0 : 65535;
        hipLaunchKernelGGL(k_shift_rows, grid_rows(K, n), dim3(256), 0, s, in + r0 * K, K,
                           out + r0 * K);
    }
    return hipGetLastError();
}

hipError_t launch_dist_sqrd(const float2 *H, int R, int K, float *P, hipStream_t s) {
    hipLaunchKernelGGL(k_dist_sqrd, dim3((K + 255) / 256), dim3(256), 0, s, H, R, K, P);
    return hipGetLastError();
}

// Order-sensitive 64-bit hash of a buffer's 32-bit words (sum over i of
// mix(w_i) * (2 i + 1) mod 2^64, one 64-bit atomic add per wave into *h,
// which the launcher zeroes first): gpuLS::demodOneSymbol's check that the
// caller's Hconj / Hsqrd still hold what firstVector exported.
__global__ void __launch_bounds__(256) k_hash_words(const unsigned *__restrict__ w, long long n,
                                                    unsigned long long *h) {
    unsigned long long acc = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        acc += ((unsigned long long)w[i] * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) *
               (unsigned long long)(2 * i + 1);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(h, acc);
}

// n 64-bit words of zeros (one vector store per thread): the capture counter
// set of the work tickets, as a kernel node -- a memset node captured by
// hipMemsetAsync replayed with a wrong value on ROCm 7.2 (the second replay
// found the set filled with a pointer-like constant, scripts/r5/capture_debug.py)
__global__ void __launch_bounds__(256) k_zero_words(unsigned long long *p, int n) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) p[i] = 0ull;
}
hipError_t launch_zero_words(unsigned long long *p, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_zero_words, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n);
    return hipGetLastError();
}

hipError_t launch_hash_words(const void *d, long long nwords, unsigned long long *h, hipStream_t s) {
    if (hipError_t e = launch_zero_words(h, 1, s); e != hipSuccess) return e;  // capturable (see above)
    if (nwords <= 0) return hipSuccess;
    long long blocks = (nwords + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_hash_words, dim3((unsigned)blocks), dim3(256), 0, s, static_cast<const unsigned *>(d),
                       nwords, h);
    return hipGetLastError();
}

}  // namespace ofdm
