// Microbenchmark: wave64 VALU issue rate on one GPU for fp64 FMA, fp64 mul+add, and int32 ops,
// with 1, 2 and 4 waves per SIMD and 1 / 4 independent dependency chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS>
__global__ void fma64(double *out, int iters, double a, double b) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) x[c] = fma(x[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.0) out[0] = s;
}

template <int CHAINS>
__global__ void int32k(unsigned *out, int iters, unsigned a) {
    unsigned x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) x[c] = (x[c] ^ a) + (x[c] >> 3);
    }
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345u) out[0] = s;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    double *d;
    hipMalloc(&d, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    printf("CUs %d, clock %d kHz\n", ncu, clk);
    for (int wps : {1, 2, 4}) {
        const int block = 256 * wps;  // one workgroup per CU: wps waves per SIMD
        auto run = [&](const char *name, auto launch, double instr_per_lane) {
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double waves = (double)ncu * block / 64;
            const double winstr = waves * instr_per_lane;
            const double per_simd_clk = winstr / (ncu * 4.0) / (ms * 1e-3 * clk * 1e3);
            printf("%-14s waves/SIMD %d: %.3f wave-instr per SIMD-clock (%.1f clk per instr)\n", name, wps,
                   per_simd_clk, 1.0 / per_simd_clk);
        };
        run("fma64 x1", [&] { hipLaunchKernelGGL(fma64<1>, dim3(ncu), dim3(block), 0, 0, d, iters, 0.999, 1e-3); },
            16.0 * iters * 1);
        run("fma64 x4", [&] { hipLaunchKernelGGL(fma64<4>, dim3(ncu), dim3(block), 0, 0, d, iters, 0.999, 1e-3); },
            16.0 * iters * 4);
        run("int32 x4 (2op)", [&] { hipLaunchKernelGGL(int32k<4>, dim3(ncu), dim3(block), 0, 0, (unsigned *)d, iters, 77u); },
            16.0 * iters * 4 * 2);
    }
    return 0;
}
