/* Does a wave's fp64 VALU issue get faster with fewer active lanes?  One wave, a chain of fp64 FMAs
 * (dependent, and 4 independent chains), timed with s_memtime under exec = 64, 16 and 1 lanes.
 * Build: hipcc --offload-arch=gfx950 -O3 exec_rate.hip -o exec_rate */
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CHAINS>
__device__ __forceinline__ double chain(double a, double b, int n) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = a + c;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fma(x[c], b, a);
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    return s;
}

__global__ void k(double *out, unsigned long long *t, double a, double b, int n, int active, int chains) {
    const int lane = threadIdx.x;
    double r = 0;
    unsigned long long t0 = 0, t1 = 0;
    if (lane < active) {
        t0 = __builtin_amdgcn_s_memtime();
        if (chains == 1) r = chain<1>(a, b, n);
        else r = chain<4>(a, b, n);
        t1 = __builtin_amdgcn_s_memtime();
    }
    if (lane < active) out[lane] = r;
    if (lane == 0) t[0] = t1 - t0;
}

int main() {
    double *out;
    unsigned long long *t, h;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&t, 8);
    const int n = 4096;
    for (int chains : {1, 4})
        for (int active : {64, 16, 1}) {
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, t, 1.0000001, 0.9999999, n, active, chains);
                hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
            }
            printf("chains %d active %2d: %.2f memtime ticks per FMA instruction\n", chains, active,
                   (double)h / ((double)n * 16 * chains));
        }
    return 0;
}
