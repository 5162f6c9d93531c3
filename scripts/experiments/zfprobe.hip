// zfprobe.hip -- diagnostic: the HBM ceiling of the ZF apply's traffic with no
// arithmetic.  Per symbol the apply (zf.hip, multiplyWithChannelInv,
// cpuLS.hpp:449-463) reads U rows of K = 1023 complex floats and writes R
// rows (subcarrier fastest); here a workgroup copies each 64-subcarrier
// column block of one symbol, out[r] = in[r % U], and the rate is reported
// over the same algorithmic bytes (U + R) * K * 8 per symbol.
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const float2 *__restrict__ in, float2 *__restrict__ out, int U, int R,
                                              int K, long long nsym) {
    const int nkb = (K + 63) / 64;
    const long long blk = blockIdx.x;
    const long long q = blk / nkb;
    const int kb = (int)(blk % nkb), w = threadIdx.x >> 6, t = threadIdx.x & 63;
    if (q >= nsym) return;
    const int k = kb * 64 + t;
    if (k >= K) return;
    const float2 *x = in + q * (long long)U * K + k;
    float2 *y = out + q * (long long)R * K + k;
    float2 v[32];
    for (int u = 0; u < U; ++u) v[u & 31] = x[(long long)u * K];
    for (int r = w; r < R; r += 4) {
        const float2 s = v[r % U & 31];
        if (NT)
            __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, s),
                                        reinterpret_cast<unsigned long long *>(y + (long long)r * K));
        else
            y[(long long)r * K] = s;
    }
}

// whole rows: a workgroup owns one symbol and writes each of its R output
// rows completely (8184 contiguous bytes, 4 waves x 4 wave-stores of 512 B)
__global__ void __launch_bounds__(256) k_rows(const float2 *__restrict__ in, float2 *__restrict__ out, int U, int R,
                                              int K, long long nsym) {
    const long long q = blockIdx.x;
    const float2 *x = in + q * (long long)U * K;
    float2 *y = out + q * (long long)R * K;
    float2 v[4][4];
    for (int r = 0; r < R; ++r) {
        if (r < U || (r % U) == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = threadIdx.x + 256 * i;
                if (k < K) v[r % 4][i] = x[(long long)(r % U) * K + k];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = threadIdx.x + 256 * i;
            if (k < K)
                __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, v[r % 4][i]),
                                            reinterpret_cast<unsigned long long *>(y + (long long)r * K + k));
        }
    }
}

double run_rows(const float2 *in, float2 *out, int U, int R, int K, long long nsym) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_rows<<<(unsigned)nsym, 256>>>(in, out, U, R, K, nsym);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) k_rows<<<(unsigned)nsym, 256>>>(in, out, U, R, K, nsym);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("U=%d R=%d nsym=%lld whole rows nt: %.3f ms  %.0f GB/s\n", U, R, nsym, ms,
           (double)(U + R) * K * 8 * nsym / (ms * 1e-3) / 1e9);
    return ms;
}

template <bool NT>
double run(const float2 *in, float2 *out, int U, int R, int K, long long nsym) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const long long blocks = nsym * ((K + 63) / 64);
    k_copy<NT><<<(unsigned)blocks, 256>>>(in, out, U, R, K, nsym);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) k_copy<NT><<<(unsigned)blocks, 256>>>(in, out, U, R, K, nsym);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("U=%d R=%d nsym=%lld %s stores: %.3f ms  %.0f GB/s\n", U, R, nsym, NT ? "nt   " : "plain", ms,
           (double)(U + R) * K * 8 * nsym / (ms * 1e-3) / 1e9);
    return ms;
}

int main() {
    const int K = 1023, R = 64;
    const long long nsym = 10000;
    float2 *in, *out;
    if (hipMalloc(&in, (size_t)nsym * 32 * K * 8) != hipSuccess) return 1;
    if (hipMalloc(&out, (size_t)nsym * R * K * 8) != hipSuccess) return 1;
    hipMemset(in, 0, (size_t)nsym * 32 * K * 8);
    for (int U : {8, 16, 32}) {
        run<false>(in, out, U, R, K, nsym);
        run<true>(in, out, U, R, K, nsym);
        run_rows(in, out, U, R, K, nsym);
    }
    return 0;
}
