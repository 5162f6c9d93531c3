// zfprobe2.hip -- diagnostic for the ZF apply's store stream (zf.hip,
// multiplyWithChannelInv, cpuLS.hpp:449-463): out[s][r][k], k < K = 1023,
// rows of 8184 B, so a 64-subcarrier column stripe (512 B) starts at an
// 8-byte (not 128-byte line) boundary and every stripe store leaves partial
// lines that a neighbouring workgroup completes later.  No arithmetic: out[s][r][k] =
// in[s][r % U][k], rate over (U + R) * K * 8 B per symbol.
//   col<K>: the apply's column stripes (workgroup = (symbol, 64 subcarriers),
//           4 waves over the rows, 8 B nt stores), K = 1023 vs K = 1024
//           (line-aligned rows): is it the partial lines?
//   flat:   workgroup = (symbol, 1/8 of the symbol's R x K outputs as one flat
//           range), 16 B nt stores, every 1 KiB wave store line-aligned
//           except at the 8 range ends.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

template <int K>
__global__ void __launch_bounds__(256) k_col(const float2 *__restrict__ in, float2 *__restrict__ out, int U, int R,
                                             long long nsym) {
    constexpr int nkb = (K + 63) / 64;
    const long long q = blockIdx.x / nkb;
    const int kb = blockIdx.x % nkb, w = threadIdx.x >> 6, t = threadIdx.x & 63;
    if (q >= nsym) return;
    const int k = kb * 64 + t;
    if (k >= K) return;
    const float2 *x = in + q * (long long)U * K + k;
    float2 *y = out + q * (long long)R * K + k;
    float2 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = u < U ? x[(long long)u * K] : float2{0.f, 0.f};
    for (int r = w; r < R; r += 4)
        __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, v[r % U]),
                                    reinterpret_cast<unsigned long long *>(y + (long long)r * K));
}

// 8 workgroups per symbol; workgroup g writes flat complex elements
// [g * R * K / 8, (g + 1) * R * K / 8) of out[s] in 16 B (2 complex) pieces
__global__ void __launch_bounds__(256) k_flat(const float2 *__restrict__ in, float2 *__restrict__ out, int U, int R,
                                              int K, long long nsym) {
    const long long q = blockIdx.x >> 3;
    const int g = blockIdx.x & 7;
    if (q >= nsym) return;
    const int n = R * K;                   // complex per symbol (even for even R)
    const int e0 = (int)((long long)n * g / 8) & ~1, e1 = g == 7 ? n : (int)((long long)n * (g + 1) / 8) & ~1;
    const float2 *x = in + q * (long long)U * K;
    float2 *y = out + q * (long long)n;
    for (int e = e0 + 2 * threadIdx.x; e < e1; e += 512) {
        const int r0 = e / K, k0 = e - r0 * K;
        const int r1 = k0 + 1 < K ? r0 : r0 + 1, k1 = k0 + 1 < K ? k0 + 1 : 0;
        const float2 a = x[(long long)(r0 % U) * K + k0], b = x[(long long)(r1 % U) * K + k1];
        f4v v = {a.x, a.y, b.x, b.y};
        __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(y + e));
    }
}

// column pieces of 2 * 64 * WK subcarriers with 16-B stores (2 subcarriers per
// lane): WK = 1: each wave a 1 KiB piece of a row, the 4 waves over the rows;
// WK = 4: the 4 waves side by side, a 4 KiB piece per row, rows in sequence.
// (Odd rows start 8 B off a 16-B boundary: those stores are misaligned.)
template <int WK>
__global__ void __launch_bounds__(256) k_col16(const float2 *__restrict__ in, float2 *__restrict__ out, int U, int R,
                                               int K, long long nsym) {
    constexpr int PK = 128 * WK;  // subcarriers per piece
    const int nkb = (K + PK - 1) / PK;
    const long long q = blockIdx.x / nkb;
    const int kb = blockIdx.x % nkb, w = threadIdx.x >> 6, t = threadIdx.x & 63;
    if (q >= nsym) return;
    const int k = kb * PK + (WK == 4 ? 128 * w : 0) + 2 * t;
    if (k >= K) return;
    const float2 *x = in + q * (long long)U * K + k;
    float2 *y = out + q * (long long)R * K + k;
    const bool pair = k + 1 < K;
    for (int r = (WK == 4 ? 0 : w); r < R; r += (WK == 4 ? 1 : 4)) {
        const float2 *xr = x + (long long)(r % U) * K;
        const float2 a = xr[0], b = pair ? xr[1] : float2{0.f, 0.f};
        if (pair) {
            f4v v = {a.x, a.y, b.x, b.y};
            __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(y + (long long)r * K));
        } else {
            __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, a),
                                        reinterpret_cast<unsigned long long *>(y + (long long)r * K));
        }
    }
}

template <typename F>
static double timed(F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipEventRecord(a);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int R = 64;
    const long long nsym = 10000;
    float2 *in, *out;
    if (hipMalloc(&in, (size_t)nsym * 32 * 1024 * 8) != hipSuccess) return 1;
    if (hipMalloc(&out, (size_t)nsym * R * 1024 * 8) != hipSuccess) return 1;
    (void)hipMemset(in, 0, (size_t)nsym * 32 * 1024 * 8);
    for (int U : {8, 16}) {  // k_col keeps U <= 16 rows in registers
        double ms = timed([&] { k_col<1023><<<(unsigned)(nsym * 16), 256>>>(in, out, U, R, nsym); });
        printf("U=%2d col stripes K=1023: %.3f ms %6.0f GB/s\n", U, ms, (double)(U + R) * 1023 * 8 * nsym / (ms * 1e-3) / 1e9);
        ms = timed([&] { k_col<1024><<<(unsigned)(nsym * 16), 256>>>(in, out, U, R, nsym); });
        printf("U=%2d col stripes K=1024: %.3f ms %6.0f GB/s\n", U, ms, (double)(U + R) * 1024 * 8 * nsym / (ms * 1e-3) / 1e9);
        ms = timed([&] { k_col16<1><<<(unsigned)(nsym * 8), 256>>>(in, out, U, R, 1023, nsym); });
        printf("U=%2d col 1 KiB 16B K=1023: %.3f ms %6.0f GB/s\n", U, ms, (double)(U + R) * 1023 * 8 * nsym / (ms * 1e-3) / 1e9);
        ms = timed([&] { k_col16<4><<<(unsigned)(nsym * 2), 256>>>(in, out, U, R, 1023, nsym); });
        printf("U=%2d col 4 KiB 16B K=1023: %.3f ms %6.0f GB/s\n", U, ms, (double)(U + R) * 1023 * 8 * nsym / (ms * 1e-3) / 1e9);
        ms = timed([&] { k_flat<<<(unsigned)(nsym * 8), 256>>>(in, out, U, R, 1023, nsym); });
        printf("U=%2d flat 16B     K=1023: %.3f ms %6.0f GB/s\n", U, ms, (double)(U + R) * 1023 * 8 * nsym / (ms * 1e-3) / 1e9);
    }
    return 0;
}
