// bwprobe.hip -- diagnostic: streaming-read bandwidth on this GPU by load
// width (8 vs 16 bytes per lane) and cache policy.  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

template <typename T, bool NT>
__global__ void __launch_bounds__(256) rd(const T *__restrict__ p, size_t n, float *out) {
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            size_t j = i + u * stride;
            if (j < n) {
                T v = NT ? __builtin_nontemporal_load(p + j) : p[j];
                acc += __builtin_bit_cast(float, (unsigned)(reinterpret_cast<const unsigned *>(&v)[0]));
            }
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

template <typename T, bool NT>
double run(const void *buf, size_t bytes, float *out, int blocks) {
    size_t n = bytes / sizeof(T);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    rd<T, NT><<<blocks, 256>>>((const T *)buf, n, out);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) rd<T, NT><<<blocks, 256>>>((const T *)buf, n, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return bytes * 5.0 / (ms * 1e-3) / 1e9;
}

int main(int argc, char **argv) {
    size_t gb = argc > 1 ? atoi(argv[1]) : 32;
    size_t bytes = gb << 30;
    void *buf; float *out;
    if (hipMalloc(&buf, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMalloc(&out, 4);
    hipMemset(buf, 0, bytes);
    for (int blocks : {2048, 8192, 32768}) {
        printf("blocks %6d  x2 %5.0f  x2nt %5.0f  x4 %5.0f  x4nt %5.0f GB/s\n", blocks,
               run<unsigned long long, false>(buf, bytes, out, blocks),
               run<unsigned long long, true>(buf, bytes, out, blocks),
               run<u4v, false>(buf, bytes, out, blocks), run<u4v, true>(buf, bytes, out, blocks));
    }
    return 0;
}
