// rfft_test.hip -- A/B build only (OFDM_AB_KNOBS): a correctness check and a
// compute-only throughput probe of the register-only 1024-point FFT
// (rfft1024.hpp) against the LDS-transpose FFT of the receiver kernels
// (wave_fft1024.hpp, hlds::row_fft_a/b).  scripts/rfft_check.py drives them.
#ifdef OFDM_AB_KNOBS
#include "launch.hpp"
#include "rfft1024.hpp"

namespace ofdm {
namespace rfftt {

namespace hl = td1024::hlds;
using td1024::row_load;

// one wave per 1024-point row, natural-order bins out
__global__ void __launch_bounds__(256) k_rfft_check(const float2 *__restrict__ in, float2 *__restrict__ out,
                                                    int nrows) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    hl::fill(lds, lds + hl::TW1S);
    __syncthreads();
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    const long long row = (long long)blockIdx.x * 4 + w;
    if (row >= nrows) return;
    float2 a[16];
    row_load<false>(in + row * 1024, t, a);
    const rfft::Consts c = rfft::make_consts(t);
    rfft::fft1024(a, t, lds, c);
#pragma unroll
    for (int j = 0; j < 16; ++j) out[row * 1024 + rfft::rfft_bin(t, j)] = a[j];
}

// each wave transforms its row ITERS times, the output (scaled by 1/32) fed
// back as the next input; NEW: register-only FFT, else the LDS-transpose one
template <int NEW, int WPE>
__global__ void __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(WPE, WPE)))
k_fft_bench(const float2 *__restrict__ in, float2 *__restrict__ out, int iters) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float2 *tw1 = lds, *tw2 = lds + hl::TW1S;
    float2 *T = lds + hl::TW1S + hl::TW2S + w * hl::TS;
    hl::fill(tw1, tw2);
    __syncthreads();
    const long long row = (long long)blockIdx.x * 8 + w;
    float2 a[16];
    row_load<false>(in + row * 1024, t, a);
    const rfft::Consts c = rfft::make_consts(t);
    for (int it = 0; it < iters; ++it) {
        if constexpr (NEW == 1) {
            rfft::fft1024(a, t, tw1, c);
        } else if constexpr (NEW == 2) {  // LDS-transpose FFT with packed-f32 halves
            float2 x[16];
            hl::row_fft_a<3>(a, t, T, tw1);
            hl::row_fft_b<3>(t, T, tw2, x);
#pragma unroll
            for (int m = 0; m < 16; ++m) a[m] = x[m];
        } else {
            float2 x[16];
            hl::row_fft_a(a, t, T, tw1);
            hl::row_fft_b(t, T, tw2, x);
#pragma unroll
            for (int m = 0; m < 16; ++m) a[m] = x[m];
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) a[m] = pk::F(pk::scale(pk::V(a[m]), 0.03125f));
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) out[row * 1024 + t + 64 * m] = a[m];
}

template <int NEW, int WPE>
hipError_t bench_launch(const float2 *in, float2 *out, long long nblocks, int iters, hipStream_t s) {
    auto k = k_fft_bench<NEW, WPE>;
    const int bytes = WPE == 2 ? 160 * 1024 : (int)hl::LDS_BYTES;  // 1 or 2 eight-wave workgroups per CU
    if (hipError_t e = opt_in_lds(reinterpret_cast<const void *>(k), bytes); e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)nblocks), dim3(512), bytes, s, in, out, iters);
    return hipGetLastError();
}

}  // namespace rfftt
}  // namespace ofdm

extern "C" int ofdm_ab_rfft_check(const void *in, void *out, int nrows, hipStream_t s) {
    using namespace ofdm;
    if (nrows <= 0) return 0;
    hipLaunchKernelGGL(rfftt::k_rfft_check, dim3((unsigned)((nrows + 3) / 4)), dim3(256),
                       (rfftt::hl::TW1S + rfftt::hl::TW2S) * sizeof(float2), s, (const float2 *)in, (float2 *)out,
                       nrows);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// rows = nblocks * 8 rows of 1024 complex in `in` and `out`
extern "C" int ofdm_ab_fft_bench(const void *in, void *out, long long nblocks, int iters, int variant, int wpe,
                                 hipStream_t s) {
    using namespace ofdm::rfftt;
    const float2 *i = (const float2 *)in;
    float2 *o = (float2 *)out;
    hipError_t e;
    if (variant == 1)
        e = wpe == 2 ? bench_launch<1, 2>(i, o, nblocks, iters, s) : bench_launch<1, 4>(i, o, nblocks, iters, s);
    else if (variant == 2)
        e = wpe == 2 ? bench_launch<2, 2>(i, o, nblocks, iters, s) : bench_launch<2, 4>(i, o, nblocks, iters, s);
    else
        e = wpe == 2 ? bench_launch<0, 2>(i, o, nblocks, iters, s) : bench_launch<0, 4>(i, o, nblocks, iters, s);
    return e == hipSuccess ? 0 : -2;
}
#endif  // OFDM_AB_KNOBS
