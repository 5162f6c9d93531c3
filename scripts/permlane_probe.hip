// diagnostic: observed semantics of __builtin_amdgcn_permlane32_swap
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *out) {
    int t = threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(100 + t, 200 + t, false, false);
    out[2 * t] = r[0];
    out[2 * t + 1] = r[1];
}
int main() {
    int *d, h[128];
    hipMalloc(&d, sizeof h);
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int t : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0=%d r1=%d\n", t, h[2 * t], h[2 * t + 1]);
    return 0;
}
