// bwprobe2.hip -- diagnostic: read bandwidth of the MRC kernel's access
// patterns (no compute).  Each wave reads 64 rows x 8 KB with 8-B lanes.
//  mode 0: wave w of block b owns symbol (8b + w), reads its rows in order
//          (the k_mrc_td1024 pattern: 4096+ streams 512 KB apart)
//  mode 1: the 8 waves of a block share one symbol, wave w reads rows
//          w, w+8, ... (a block streams 64 KB contiguous per step)
//  mode 2: grid-stride contiguous 8-B loads (reference)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;
template <int MODE>
__global__ void __launch_bounds__(512) rd(const u64 *__restrict__ p, long long nsym, float *out) {
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float acc = 0.f;
    if (MODE == 0) {
        for (long long q = (long long)blockIdx.x * 8 + w; q < nsym; q += (long long)gridDim.x * 8) {
            const u64 *s = p + q * 65536;  // 512 KB per symbol (u64 = 8 B)
            for (int r = 0; r < 64; ++r) {
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    u64 v = __builtin_nontemporal_load(s + r * 1024 + t + 64 * m);
                    acc += __builtin_bit_cast(float, (unsigned)v);
                }
            }
        }
    } else if (MODE == 1) {
        for (long long q = blockIdx.x; q < nsym; q += gridDim.x) {
            const u64 *s = p + q * 65536;
            for (int r = w; r < 64; r += 8) {
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    u64 v = __builtin_nontemporal_load(s + r * 1024 + t + 64 * m);
                    acc += __builtin_bit_cast(float, (unsigned)v);
                }
            }
        }
    } else {
        const long long n = nsym * 65536;
        for (long long i = (long long)blockIdx.x * 512 + threadIdx.x; i < n; i += (long long)gridDim.x * 512) {
            u64 v = __builtin_nontemporal_load(p + i);
            acc += __builtin_bit_cast(float, (unsigned)v);
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}
template <int MODE>
double run(const u64 *p, long long nsym, float *out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    rd<MODE><<<blocks, 512>>>(p, nsym, out);
    hipEventRecord(a);
    for (int i = 0; i < 3; ++i) rd<MODE><<<blocks, 512>>>(p, nsym, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return nsym * 524288.0 * 3 / (ms * 1e-3) / 1e9;
}
int main() {
    const long long nsym = 65536;  // 32 GiB
    u64 *p; float *out;
    if (hipMalloc(&p, nsym * 524288) != hipSuccess) return 1;
    hipMalloc(&out, 4);
    hipMemset(p, 0, nsym * 524288);
    for (int blocks : {512, 1024, 4096})
        printf("blocks %5d: per-wave symbol %5.0f  block-shared symbol %5.0f  grid-stride %5.0f GB/s\n",
               blocks, run<0>(p, nsym, out, blocks), run<1>(p, nsym, out, blocks), run<2>(p, nsym, out, blocks));
}
