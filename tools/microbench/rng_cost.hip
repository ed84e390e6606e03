// Cost of one 53-bit uniform: the transport's Philox4x32-10 (grm_device.h uniform) against a
// SplitMix64 counter hash -- wave-instruction time measured with HIP events over a full grid.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../cuda-grmonty_amd/csrc/grm_device.h"
using namespace grm;

__device__ __forceinline__ double sm_uniform(uint64_t key, uint32_t &ctr) {
    uint64_t z = key + 0x9E3779B97F4A7C15ull * (uint64_t)(++ctr);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)((z >> 11) + 1) * (1.0 / 9007199254740992.0);
}

__global__ void k_philox(double *out, int n) {
    Rng r;
    r.k0 = 123; r.k1 = 0; r.id = blockIdx.x * 512ull + threadIdx.x; r.ctr = 0; r.ctr_hi = 0;
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += uniform(r);
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

__global__ void k_splitmix(double *out, int n) {
    uint64_t key = splitmix64(blockIdx.x * 512ull + threadIdx.x);
    uint32_t ctr = 0;
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += sm_uniform(key, ctr);
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 2, n = 20000;
    double *d;
    hipMalloc(&d, blocks * 512 * sizeof(double));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) {
        float ms[2];
        for (int k = 0; k < 2; ++k) {
            hipEventRecord(a);
            if (k == 0) hipLaunchKernelGGL(k_philox, dim3(blocks), dim3(512), 0, 0, d, n);
            else hipLaunchKernelGGL(k_splitmix, dim3(blocks), dim3(512), 0, 0, d, n);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms[k], a, b);
        }
        const double waves = blocks * 8.0, simds = 1024.0;
        for (int k = 0; k < 2; ++k)
            printf("%s: %.2f ms, %.1f SIMD-cycles per wave-draw (2.4 GHz)\n", k ? "splitmix64" : "philox4x32-10", ms[k],
                   ms[k] * 1e-3 * 2.4e9 * simds / (waves * n));
    }
    return 0;
}
