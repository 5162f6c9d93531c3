// wrprobe.hip -- diagnostic: what HBM sustains for WRITE-dominated streams,
// the traffic of the zero-forcing apply (zf.hip, multiplyWithChannelInv,
// cpuLS.hpp:449-463: per symbol U input rows read, R = 64 output rows
// written, 80 % of the bytes stores at U = 16).  Each kernel moves a fixed
// byte count with no arithmetic; rates are bytes moved / kernel time.
//   write16 / write8: pure stores, 16 or 8 B per lane, nontemporal, each
//                     workgroup a contiguous 64 KiB span per iteration
//   read16:           pure loads of the same size (reference)
//   rw16_1to4:        the apply's mix: per 5 units, 1 read + 4 written
//                     (each workgroup reads one 2 KiB piece, writes four)
//   rows16:           the apply's shape with whole 8 KiB rows, 16 B stores:
//                     a workgroup per symbol reads U rows and writes R rows
// usage: ./wrprobe  (prints one line per variant)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

template <int VB>
__global__ void __launch_bounds__(256) k_write(char *__restrict__ out, long long nbytes, int iters) {
    // grid-stride over 64 KiB spans: each workgroup writes 64 KiB contiguous per step
    const long long span = 256LL * VB * (65536 / (256 * VB));
    for (long long base = (long long)blockIdx.x * span; base < nbytes; base += (long long)gridDim.x * span) {
#pragma unroll 4
        for (int i = 0; i < 65536 / (256 * VB); ++i) {
            const long long off = base + ((long long)i * 256 + threadIdx.x) * VB;
            if (VB == 16) {
                f4v v = {1.f, 2.f, 3.f, (float)iters};
                __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(out + off));
            } else {
                unsigned long long v = 0x3f8000003f800000ull + iters;
                __builtin_nontemporal_store(v, reinterpret_cast<unsigned long long *>(out + off));
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_read(const char *__restrict__ in, long long nbytes, float *sink) {
    const long long span = 65536;
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    for (long long base = (long long)blockIdx.x * span; base < nbytes; base += (long long)gridDim.x * span) {
#pragma unroll 4
        for (int i = 0; i < 16; ++i) {
            const long long off = base + ((long long)i * 256 + threadIdx.x) * 16;
            acc += __builtin_nontemporal_load(reinterpret_cast<const f4v *>(in + off));
        }
    }
    if (acc.x == 1234.5f) sink[0] = acc.y;
}

// per 10 KiB unit: read 2 KiB, write 8 KiB (the apply's 1 : 4 at U = 16, R = 64)
__global__ void __launch_bounds__(128) k_rw(const char *__restrict__ in, char *__restrict__ out, long long units) {
    for (long long u = blockIdx.x; u < units; u += gridDim.x) {
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(in + u * 2048 + threadIdx.x * 16));
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(out + u * 8192 + j * 2048 + threadIdx.x * 16));
    }
}

// the apply's shape: symbol q reads U rows of K complex (8184 B) and writes R rows;
// 256 threads, 16 B per lane (a row = 511.5 float4: 512 lanes cover it, the
// last lane of each row skipped)
__global__ void __launch_bounds__(256) k_rows16(const float2 *__restrict__ in, float2 *__restrict__ out, int U,
                                                int R, int K, long long nsym) {
    for (long long q = blockIdx.x; q < nsym; q += gridDim.x) {
        const float2 *x = in + q * (long long)U * K;
        float2 *y = out + q * (long long)R * K;
        for (int r = 0; r < R; ++r) {
            const float2 *xr = x + (long long)(r % U) * K;
            float2 *yr = y + (long long)r * K;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = 2 * (threadIdx.x + 256 * h);
                if (k + 1 < K) {
                    float4 v;
                    v.x = xr[k].x; v.y = xr[k].y; v.z = xr[k + 1].x; v.w = xr[k + 1].y;
                    // rows are 8184 B apart: 16 B stores are 8 B aligned only on odd rows
                    __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, float2{v.x, v.y}),
                                                reinterpret_cast<unsigned long long *>(yr + k));
                    __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, float2{v.z, v.w}),
                                                reinterpret_cast<unsigned long long *>(yr + k + 1));
                } else if (k < K) {
                    __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, xr[k]),
                                                reinterpret_cast<unsigned long long *>(yr + k));
                }
            }
        }
    }
}

template <typename F>
static double timed(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const long long NB = 5LL << 30;  // 5 GiB: the apply's output at U = 16, 10 000 symbols
    char *buf = nullptr, *src = nullptr;
    float *sink = nullptr;
    if (hipMalloc(&buf, NB) != hipSuccess || hipMalloc(&src, NB / 4) != hipSuccess ||
        hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    hipMemset(buf, 0, NB);
    hipMemset(src, 0, NB / 4);
    int cus = 256;
    for (int per_cu : {2, 4, 8}) {
        const int grid = cus * per_cu;
        double ms = timed([&] { k_write<16><<<grid, 256>>>(buf, NB, 1); });
        printf("write16 nt   grid=%5d: %.3f ms %7.0f GB/s\n", grid, ms, NB / (ms * 1e-3) / 1e9);
        ms = timed([&] { k_write<8><<<grid, 256>>>(buf, NB, 1); });
        printf("write8  nt   grid=%5d: %.3f ms %7.0f GB/s\n", grid, ms, NB / (ms * 1e-3) / 1e9);
        ms = timed([&] { k_read<<<grid, 256>>>(buf, NB, sink); });
        printf("read16  nt   grid=%5d: %.3f ms %7.0f GB/s\n", grid, ms, NB / (ms * 1e-3) / 1e9);
    }
    const long long units = NB / 8192;
    for (int grid : {1024, 2048, 4096}) {
        double ms = timed([&] { k_rw<<<grid, 128>>>(src, buf, units); });
        printf("rw 1:4 nt    grid=%5d: %.3f ms %7.0f GB/s (read %.2f GB, written %.2f GB)\n", grid, ms,
               units * 10240.0 / (ms * 1e-3) / 1e9, units * 2048 / 1e9, units * 8192 / 1e9);
    }
    const int U = 16, R = 64, K = 1023;
    const long long nsym = 10000;
    for (int grid : {1024, 2048, 10000}) {
        double ms = timed([&] {
            k_rows16<<<grid, 256>>>(reinterpret_cast<const float2 *>(src), reinterpret_cast<float2 *>(buf), U, R, K,
                                    nsym);
        });
        printf("rows (apply shape U=16 R=64, 10k symbols) grid=%5d: %.3f ms %7.0f GB/s algorithmic\n", grid, ms,
               (double)(U + R) * K * 8 * nsym / (ms * 1e-3) / 1e9);
    }
    return 0;
}
