// fft_synth.hip -- generic batched row FFT (Stockham in LDS) and the synthetic
// OFDM frame generator / hard-decision checker used by tests and bench.
//
// The FFT replaces the reference's cuFFT batch (gpuLS::batchedFFT,
// gpuLS.cu:343-349; cufftPlan1d + cufftExecC2C, gpuLS.cu:377-381) and FFTW's
// fftOneRow (cpuLS.hpp:165-174): unnormalised forward C2C, sign -1.
#include "common.hpp"
#include "launch.hpp"

namespace ofdm {

template <int LOG2C, bool INV>
__global__ void __launch_bounds__(256) k_fft_rows(const float2 *__restrict__ in, long long in_stride,
                                                  int in_off, float2 *out, long long out_stride,
                                                  int out_off, float scale) {
    constexpr int C = 1 << LOG2C;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *a = lds, *b = lds + C;
    const long long row = blockIdx.x;
    const float2 *src = in + row * in_stride + in_off;
    for (int i = threadIdx.x; i < C; i += blockDim.x) a[i] = src[i];
    __syncthreads();
    float2 *res = stockham_lds<LOG2C, INV>(a, b);
    float2 *dst = out + row * out_stride + out_off;
    for (int i = threadIdx.x; i < C; i += blockDim.x) {
        float2 v = res[i];
        dst[i] = float2{v.x * scale, v.y * scale};
    }
}

template <int LOG2C>
static hipError_t fft_rows_t(const float2 *in, long long in_stride, int in_off, float2 *out,
                             long long out_stride, int out_off, long long nrows, bool inverse,
                             float scale, hipStream_t s) {
    constexpr int C = 1 << LOG2C;
    const int threads = C / 4 < 256 ? (C / 4 < 64 ? 64 : C / 4) : 256;
    const size_t lds = 2 * C * sizeof(float2);
    // grid.x limit is 2^31-1; split very large batches
    const long long maxg = 1ll << 30;
    for (long long r0 = 0; r0 < nrows; r0 += maxg) {
        const long long n = nrows - r0 < maxg ? nrows - r0 : maxg;
        if (inverse)
            hipLaunchKernelGGL((k_fft_rows<LOG2C, true>), dim3((unsigned)n), dim3(threads), lds, s,
                               in + r0 * in_stride, in_stride, in_off, out + r0 * out_stride,
                               out_stride, out_off, scale);
        else
            hipLaunchKernelGGL((k_fft_rows<LOG2C, false>), dim3((unsigned)n), dim3(threads), lds, s,
                               in + r0 * in_stride, in_stride, in_off, out + r0 * out_stride,
                               out_stride, out_off, scale);
    }
    return hipGetLastError();
}

hipError_t launch_fft_rows(const float2 *in, long long in_stride, int in_off, float2 *out,
                           long long out_stride, int out_off, long long nrows, int C,
                           bool inverse, float scale, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    switch (C) {
#define OFDM_FFT_CASE(L) \
    case 1 << L: return fft_rows_t<L>(in, in_stride, in_off, out, out_stride, out_off, nrows, inverse, scale, s);
        OFDM_FFT_CASE(2) OFDM_FFT_CASE(3) OFDM_FFT_CASE(4) OFDM_FFT_CASE(5) OFDM_FFT_CASE(6)
        OFDM_FFT_CASE(7) OFDM_FFT_CASE(8) OFDM_FFT_CASE(9) OFDM_FFT_CASE(10) OFDM_FFT_CASE(11)
        OFDM_FFT_CASE(12)
#undef OFDM_FFT_CASE
    default: return launch_fft_any(in, in_stride, in_off, out, out_stride, out_off, nrows, C, inverse, scale, s);
    }
}

// --------------------------------------------------------------------------
// Synthetic frames (SURVEY.md 8(d) "Synthetic inputs", RX convention of
// 8(a) item 7): per frame f, antenna r, subcarrier j:
//   H ~ CN(0,1), x_0 = X (pilot), x_s = QPSK (+-1/sqrt2 +- i/sqrt2), s >= 1
//   Y[j+1] = H x, Y[0] = 0;  y = IFFT_C(Y)/sqrt(C) + CN(0, noise^2), with a
//   cyclic prefix of `prefix` samples (time domain), or y = Y + noise (freq).
// Everything is a pure function of (seed, global frame, symbol, antenna, bin)
// so any shard of a batch can be regenerated independently.
// --------------------------------------------------------------------------
__device__ __forceinline__ float2 synth_channel(uint64_t seed, long long fg, int r, int j) {
    const float2 g = gauss2(hash4(seed, 1, (uint64_t)fg, ((uint64_t)r << 32) | (uint32_t)j));
    return {g.x * 0.70710678118654752f, g.y * 0.70710678118654752f};
}
__device__ __forceinline__ uint32_t synth_bits(uint64_t seed, long long fg, int s, int j) {
    return (uint32_t)hash4(seed, 2, (uint64_t)fg, ((uint64_t)s << 32) | (uint32_t)j) & 3u;
}
__device__ __forceinline__ float2 qpsk(uint32_t bits) {
    const float a = 0.70710678118654752f;
    return {(bits & 1u) ? a : -a, (bits & 2u) ? a : -a};
}

template <int LOG2C>
__global__ void __launch_bounds__(256) k_synth(float2 *iq, int S, int R, int prefix,
                                               const float2 *__restrict__ X, uint64_t seed,
                                               long long frame0, float noise_std, int freq_domain,
                                               int r0) {
    constexpr int C = 1 << LOG2C;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *a = lds, *b = lds + C;
    // one block per (frame, symbol, antenna) row
    const long long row = blockIdx.x;
    const int r = (int)(row % R);
    const long long fs = row / R;
    const int s = (int)(fs % S);
    const long long f = fs / S;
    const long long fg = frame0 + f;
    const int rg = r0 + r;
    const int Cp = freq_domain ? C : C + prefix;
    float2 *dst = iq + row * Cp;
    for (int bin = threadIdx.x; bin < C; bin += blockDim.x) {
        float2 v{0.f, 0.f};
        if (bin > 0) {
            const int j = bin - 1;
            const float2 h = synth_channel(seed, fg, rg, j);
            const float2 x = s == 0 ? X[j] : qpsk(synth_bits(seed, fg, s, j));
            v = cmul(h, x);
        }
        a[bin] = v;
    }
    __syncthreads();
    const float ns = noise_std * 0.70710678118654752f;
    const uint64_t nkey = (((uint64_t)fg * (uint64_t)S + (uint64_t)s) << 20) ^ (uint64_t)rg;
    if (freq_domain) {
        for (int n = threadIdx.x; n < C; n += blockDim.x) {
            const float2 g = gauss2(hash4(seed, 3, nkey, (uint64_t)n));
            dst[n] = float2{a[n].x + ns * g.x, a[n].y + ns * g.y};
        }
        return;
    }
    float2 *res = stockham_lds<LOG2C, true>(a, b);
    const float sc = rsqrtf((float)C);
    for (int n = threadIdx.x; n < C; n += blockDim.x) {
        const float2 g = gauss2(hash4(seed, 3, nkey, (uint64_t)n));
        res[n] = float2{res[n].x * sc + ns * g.x, res[n].y * sc + ns * g.y};
    }
    __syncthreads();
    for (int n = threadIdx.x; n < C + prefix; n += blockDim.x)
        dst[n] = n < prefix ? res[C - prefix + n] : res[n - prefix];
}

template <int LOG2C>
static hipError_t synth_t(float2 *iq, long long nframes, int S, int R, int prefix,
                          const float2 *X, uint64_t seed, long long frame0, float noise_std,
                          int freq_domain, int r0, hipStream_t s) {
    constexpr int C = 1 << LOG2C;
    const int threads = C / 4 < 256 ? (C / 4 < 64 ? 64 : C / 4) : 256;
    const size_t lds = 2 * C * sizeof(float2);
    const long long rows = nframes * S * R;
    const long long maxg = 1ll << 30;
    const long long Cp = freq_domain ? C : C + prefix;
    for (long long q0 = 0; q0 < rows; q0 += maxg) {
        // chunk boundaries must be whole frames for the index math
        long long n = rows - q0 < maxg ? rows - q0 : maxg;
        const long long frame_rows = (long long)S * R;
        n = (n / frame_rows) * frame_rows;
        hipLaunchKernelGGL(k_synth<LOG2C>, dim3((unsigned)n), dim3(threads), lds, s, iq + q0 * Cp, S,
                           R, prefix, X, seed, frame0 + q0 / frame_rows, noise_std, freq_domain, r0);
    }
    return hipGetLastError();
}

// Any other C (fft_any.hip sizes): the same frames in three passes over the
// output rows -- the bins H x into row[prefix + b] (k_synth_bins), the
// inverse FFT in place with the 1/sqrt(C) scale, then the noise and the
// cyclic prefix (k_synth_noise_cp, one workgroup per row: the prefix copies
// the noisy tail, as k_synth does).  The frequency-domain form adds its noise
// in the first pass.
__global__ void __launch_bounds__(256) k_synth_bins(float2 *iq, long long rows, int S, int R, int C, int prefix,
                                                    const float2 *__restrict__ X, uint64_t seed, long long frame0,
                                                    float noise_std, int freq_domain, int r0) {
    const int Cp = freq_domain ? C : C + prefix;
    const float ns = noise_std * 0.70710678118654752f;
    for (long long row = blockIdx.y; row < rows; row += gridDim.y) {
        const int r = (int)(row % R);
        const long long fs = row / R;
        const int s = (int)(fs % S);
        const long long fg = frame0 + fs / S;
        const int rg = r0 + r;
        const uint64_t nkey = (((uint64_t)fg * (uint64_t)S + (uint64_t)s) << 20) ^ (uint64_t)rg;
        float2 *dst = iq + row * Cp + (freq_domain ? 0 : prefix);
        for (int bin = blockIdx.x * blockDim.x + threadIdx.x; bin < C; bin += gridDim.x * blockDim.x) {
            float2 v{0.f, 0.f};
            if (bin > 0) {
                const int j = bin - 1;
                const float2 x = s == 0 ? X[j] : qpsk(synth_bits(seed, fg, s, j));
                v = cmul(synth_channel(seed, fg, rg, j), x);
            }
            if (freq_domain) {
                const float2 g = gauss2(hash4(seed, 3, nkey, (uint64_t)bin));
                v = float2{v.x + ns * g.x, v.y + ns * g.y};
            }
            dst[bin] = v;
        }
    }
}

__global__ void __launch_bounds__(256) k_synth_noise_cp(float2 *iq, long long rows, int S, int R, int C, int prefix,
                                                        uint64_t seed, long long frame0, float noise_std, int r0) {
    const float ns = noise_std * 0.70710678118654752f;
    for (long long row = blockIdx.x; row < rows; row += gridDim.x) {
        const int r = (int)(row % R);
        const long long fs = row / R;
        const int s = (int)(fs % S);
        const long long fg = frame0 + fs / S;
        const uint64_t nkey = (((uint64_t)fg * (uint64_t)S + (uint64_t)s) << 20) ^ (uint64_t)(r0 + r);
        float2 *dst = iq + row * (C + prefix);
        for (int n = threadIdx.x; n < C; n += blockDim.x) {
            const float2 g = gauss2(hash4(seed, 3, nkey, (uint64_t)n));
            const float2 v = dst[prefix + n];
            dst[prefix + n] = float2{v.x + ns * g.x, v.y + ns * g.y};
        }
        __syncthreads();  // the prefix copies the noisy tail
        for (int n = threadIdx.x; n < prefix; n += blockDim.x) dst[n] = dst[C + n];
        __syncthreads();
    }
}

static hipError_t synth_any(float2 *iq, long long nframes, int S, int R, int C, int prefix, const float2 *X,
                            uint64_t seed, long long frame0, float noise_std, int freq_domain, int r0,
                            hipStream_t s) {
    if (!fft_any_supported(C)) return hipErrorInvalidValue;
    const long long rows = nframes * S * R;
    const unsigned gx = (unsigned)((C + 255) / 256);
    const unsigned gy = (unsigned)(rows < 65535 ? rows : 65535);
    hipLaunchKernelGGL(k_synth_bins, dim3(gx, gy), dim3(256), 0, s, iq, rows, S, R, C, prefix, X, seed, frame0,
                       noise_std, freq_domain, r0);
    if (freq_domain) return hipGetLastError();
    const hipError_t e = launch_fft_any(iq, C + prefix, prefix, iq, C + prefix, prefix, rows, C, true,
                                        1.0f / sqrtf((float)C), s);
    if (e != hipSuccess) return e;
    const unsigned g = (unsigned)(rows < 16384 ? rows : 16384);
    hipLaunchKernelGGL(k_synth_noise_cp, dim3(g), dim3(256), 0, s, iq, rows, S, R, C, prefix, seed, frame0,
                       noise_std, r0);
    return hipGetLastError();
}

hipError_t launch_synth(float2 *iq, long long nframes, int S, int R, int C, int prefix,
                        const float2 *X, uint64_t seed, long long frame0, float noise_std,
                        int freq_domain, int r0, hipStream_t s) {
    if (nframes <= 0) return hipSuccess;
    switch (C) {
#define OFDM_SYN_CASE(L) \
    case 1 << L: return synth_t<L>(iq, nframes, S, R, prefix, X, seed, frame0, noise_std, freq_domain, r0, s);
        OFDM_SYN_CASE(2) OFDM_SYN_CASE(3) OFDM_SYN_CASE(4) OFDM_SYN_CASE(5) OFDM_SYN_CASE(6)
        OFDM_SYN_CASE(7) OFDM_SYN_CASE(8) OFDM_SYN_CASE(9) OFDM_SYN_CASE(10) OFDM_SYN_CASE(11)
        OFDM_SYN_CASE(12)
#undef OFDM_SYN_CASE
    default: return synth_any(iq, nframes, S, R, C, prefix, X, seed, frame0, noise_std, freq_domain, r0, s);
    }
}

__global__ void __launch_bounds__(256) k_count_errors(const float2 *__restrict__ out, long long total,
                                                      int S, int K, uint64_t seed, long long frame0,
                                                      unsigned long long *errors) {
    unsigned long long local = 0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
        const int k = (int)(e % K);
        const long long q = e / K;  // data symbol index
        const long long f = q / (S - 1);
        const int s = 1 + (int)(q % (S - 1));
        const int j = out_src(k, K);
        const uint32_t bits = synth_bits(seed, frame0 + f, s, j);
        const float2 v = out[e];
        const bool ok = ((v.x > 0.f) == ((bits & 1u) != 0)) && ((v.y > 0.f) == ((bits & 2u) != 0));
        local += ok ? 0 : 1;
    }
    // wave reduce then one atomic per wave
    for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(errors, local);
}

hipError_t launch_count_errors(const float2 *out, long long nframes, int S, int C, uint64_t seed,
                               long long frame0, unsigned long long *errors, hipStream_t s) {
    const long long total = nframes * (S - 1) * (long long)(C - 1);
    if (total <= 0) return hipSuccess;
    long long blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_count_errors, dim3((unsigned)blocks), dim3(256), 0, s, out, total, S, C - 1,
                       seed, frame0, errors);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// HBM probes of the box (bench.py's roofline.box_*): a streaming float4 copy
// and a streaming float4 read (summed; one float per thread written so the
// loads are kept) over `n4` float4s.  Each wave moves 16 KiB chunks -- 16
// dwordx4 loads per lane issued before any is used (16 KiB in flight per
// wave, 32 waves per CU) -- chunk c + grid waves next, non-temporal like the
// receivers' IQ stream; the tail (< 16 KiB) by single loads.  This is the
// ceiling of the receivers' access pattern (contiguous multi-KiB pieces per
// wave) on this box, measured in the same process right after the timed
// loop.
// ---------------------------------------------------------------------------
constexpr int PROBE_TPB = 256, PROBE_U = 16;
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float4 *p) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
    return float4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void st_nt(float4 v, float4 *p) {
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v *>(p));
}

__global__ void __launch_bounds__(PROBE_TPB) k_hbm_copy(const float4 *__restrict__ src, float4 *__restrict__ dst,
                                                        long long n4) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * PROBE_TPB + threadIdx.x) >> 6;
    const long long nwaves = (long long)gridDim.x * (PROBE_TPB / 64);
    const long long chunk = 64 * PROBE_U, nchunks = n4 / chunk;
    for (long long c = wave; c < nchunks; c += nwaves) {
        const float4 *s = src + c * chunk + lane;
        float4 *d = dst + c * chunk + lane;
        float4 v[PROBE_U];
#pragma unroll
        for (int u = 0; u < PROBE_U; ++u) v[u] = ld_nt(s + 64 * u);
#pragma unroll
        for (int u = 0; u < PROBE_U; ++u) st_nt(v[u], d + 64 * u);
    }
    for (long long i = nchunks * chunk + (long long)blockIdx.x * PROBE_TPB + threadIdx.x; i < n4;
         i += (long long)gridDim.x * PROBE_TPB)
        dst[i] = src[i];
}

__global__ void __launch_bounds__(PROBE_TPB) k_hbm_read(const float4 *__restrict__ src, float *__restrict__ sink,
                                                        long long n4) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * PROBE_TPB + threadIdx.x) >> 6;
    const long long nwaves = (long long)gridDim.x * (PROBE_TPB / 64);
    const long long chunk = 64 * PROBE_U, nchunks = n4 / chunk;
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long c = wave; c < nchunks; c += nwaves) {
        const float4 *s = src + c * chunk + lane;
        float4 v[PROBE_U];
#pragma unroll
        for (int u = 0; u < PROBE_U; ++u) v[u] = ld_nt(s + 64 * u);
#pragma unroll
        for (int u = 0; u < PROBE_U; ++u) {
            acc.x += v[u].x;
            acc.y += v[u].y;
            acc.z += v[u].z;
            acc.w += v[u].w;
        }
    }
    for (long long i = nchunks * chunk + (long long)blockIdx.x * PROBE_TPB + threadIdx.x; i < n4;
         i += (long long)gridDim.x * PROBE_TPB) {
        const float4 a = src[i];
        acc.x += a.x;
        acc.y += a.y;
        acc.z += a.z;
        acc.w += a.w;
    }
    sink[(long long)blockIdx.x * PROBE_TPB + threadIdx.x] = (acc.x + acc.y) + (acc.z + acc.w);
}

hipError_t launch_hbm_probe(int mode, const void *src, void *dst, long long n4, hipStream_t s) {
    if (n4 <= 0) return hipSuccess;
    const int blocks = 256 * 4;  // 4 workgroups of 256 threads per CU (16 waves, 256 KiB in flight)
    if (mode == 0)
        hipLaunchKernelGGL(k_hbm_copy, dim3(blocks), dim3(PROBE_TPB), 0, s, static_cast<const float4 *>(src),
                           static_cast<float4 *>(dst), n4);
    else
        hipLaunchKernelGGL(k_hbm_read, dim3(blocks), dim3(PROBE_TPB), 0, s, static_cast<const float4 *>(src),
                           static_cast<float *>(dst), n4);
    return hipGetLastError();
}

}  // namespace ofdm
