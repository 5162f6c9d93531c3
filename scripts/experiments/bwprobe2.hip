// bwprobe2.hip -- diagnostic: read bandwidth of the MRC kernel's access
// patterns (no compute).  Each wave reads 64 rows x 8 KB with 8-B lanes.
//  mode 0: wave w of block b owns symbol (8b + w), reads its rows in order
//          (the k_mrc_td1024 pattern: 4096+ streams 512 KB apart)
//  mode 1: the 8 waves of a block share one symbol, wave w reads rows
//          w, w+8, ... (a block streams 64 KB contiguous per step)
//  mode 2: grid-stride contiguous 8-B loads (reference)
//  mode 3: one symbol per wave, one-shot grid (nsym/8 blocks), XCD-grouped
//          block remap, 78.9 KB dynamic LDS (the k_mrc_td1024_w8 skeleton)
//  mode 4: as 3 without the remap; mode 5: as 3 without the LDS
//  mode 6: as 3 plus 8 KB of stores per wave at the end (pitch 1023 float2)
//  mode 7: pitch 1024 (line aligned); 8: pitch 1024 with dwordx4; 9: mode 6 with nt stores
//  mode 10: mode 0 (persistent) with the stores; 11: mode 6 into a 512 KB (L2-resident) region
//  mode 12: mode 3 + one contiguous 64 KB float4 burst per workgroup after a barrier
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;
template <int MODE>
__global__ void __launch_bounds__(512) rd(const u64 *__restrict__ p, long long nsym, float *out) {
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    float acc = 0.f;
    if (MODE == 0 || MODE == 10) {
        for (long long q = (long long)blockIdx.x * 8 + w; q < nsym; q += (long long)gridDim.x * 8) {
            const u64 *s = p + q * 65536;  // 512 KB per symbol (u64 = 8 B)
            for (int r = 0; r < 64; ++r) {
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    u64 v = __builtin_nontemporal_load(s + r * 1024 + t + 64 * m);
                    acc += __builtin_bit_cast(float, (unsigned)v);
                }
            }
            if (MODE == 10) {
                float2 *o = reinterpret_cast<float2 *>(out) + 16 + q * 1023;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int j = t + 64 * k;
                    if (j < 1023) o[j] = float2{acc, (float)k};
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
    } else if (MODE >= 3 && MODE != 10) {
        extern __shared__ float lds[];
        const long long pb = blockIdx.x, per_xcd = gridDim.x / 8;
        const long long lb = MODE == 4 ? pb : (pb & 7) * per_xcd + (pb >> 3);
        const long long q = lb * 8 + w;
        if (q < nsym) {
            const u64 *s = p + q * 65536;
            for (int r = 0; r < 64; ++r) {
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    u64 v = __builtin_nontemporal_load(s + r * 1024 + t + 64 * m);
                    acc += __builtin_bit_cast(float, (unsigned)v);
                }
            }
        }
        if (MODE != 5 && acc == 1234.5f) lds[threadIdx.x] = acc;
        if (MODE == 12) {  // the workgroup's 8 x 8184 B written as one contiguous burst of float4
            __syncthreads();
            const long long base = (long long)lb * 8 * 1023 * 8 / 16;  // float4 index
            float4 *o4 = reinterpret_cast<float4 *>(out) + 16 + base;
            for (int i = threadIdx.x; i < 8 * 1023 / 2; i += 512) o4[i] = float4{acc, (float)i, acc, 1.f};
        }
        if (MODE >= 6 && MODE != 12 && q < nsym) {  // 8 KB of output per wave, like the MRC epilogue
            const int pitch = (MODE == 7 || MODE == 8) ? 1024 : 1023;
            float2 *o = reinterpret_cast<float2 *>(out) + 16 + (MODE == 11 ? (q & 63) : q) * pitch;
            if (MODE == 8) {
                float4 *o4 = reinterpret_cast<float4 *>(o);
#pragma unroll
                for (int k = 0; k < 8; ++k) o4[t + 64 * k] = float4{acc, (float)k, acc, 1.f};
            } else {
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int j = t + 64 * k;
                    if (j < 1023) {
                        if (MODE == 9) __builtin_nontemporal_store(__builtin_bit_cast(u64, float2{acc, (float)k}), reinterpret_cast<u64 *>(o + j));
                        else o[j] = float2{acc, (float)k};
                    }
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
    size_t lds = 0;
    if (MODE >= 11 || (MODE >= 3 && MODE < 10)) { blocks = (int)(nsym / 8); lds = MODE == 5 ? 0 : 80768; }
    rd<MODE><<<blocks, 512, lds>>>(p, nsym, out);
    hipEventRecord(a);
    for (int i = 0; i < 3; ++i) rd<MODE><<<blocks, 512, lds>>>(p, nsym, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return nsym * 524288.0 * 3 / (ms * 1e-3) / 1e9;
}
__global__ void fill_random(u64 *p, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        u64 z = (u64)i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}
int main() {
    const long long nsym = 65536;  // 32 GiB
    u64 *p; float *out;
    if (hipMalloc(&p, nsym * 524288) != hipSuccess) return 1;
    hipMalloc(&out, (size_t)nsym * 8192 + 8192);
    for (int fill = 0; fill < 2; ++fill) {
        if (fill == 0) hipMemset(p, 0, nsym * 524288);
        else fill_random<<<4096, 256>>>(p, nsym * 65536);
        hipDeviceSynchronize();
        for (int blocks : {512, 1024, 4096})
            printf("%s blocks %5d: per-wave symbol %5.0f  block-shared symbol %5.0f  grid-stride %5.0f GB/s\n",
                   fill ? "random" : "zeros ", blocks, run<0>(p, nsym, out, blocks), run<1>(p, nsym, out, blocks),
                   run<2>(p, nsym, out, blocks));
        printf("%s one-shot grid: remap+lds %5.0f  lds only %5.0f  remap only %5.0f GB/s\n",
               fill ? "random" : "zeros ", run<3>(p, nsym, out, 0), run<4>(p, nsym, out, 0), run<5>(p, nsym, out, 0));
        printf("%s +stores: pitch1023 %5.0f  pitch1024 %5.0f  pitch1024 x4 %5.0f  pitch1023 nt %5.0f GB/s\n",
               fill ? "random" : "zeros ", run<6>(p, nsym, out, 0), run<7>(p, nsym, out, 0), run<8>(p, nsym, out, 0),
               run<9>(p, nsym, out, 0));
        printf("%s persistent 1024 blocks +stores %5.0f   one-shot stores into 512 KB %5.0f   64 KB block burst %5.0f GB/s\n",
               fill ? "random" : "zeros ", run<10>(p, nsym, out, 1024), run<11>(p, nsym, out, 0),
               run<12>(p, nsym, out, 0));
    }
}
