#include <hip/hip_runtime.h>
__global__ void k(unsigned *o) {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 4, 2)" : "=s"(v));
    unsigned w;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(w));
    unsigned cu;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 8, 4)" : "=s"(cu));
    if ((threadIdx.x & 63) == 0) { o[blockIdx.x * 32 + (threadIdx.x >> 6) * 4] = v; o[blockIdx.x * 32 + (threadIdx.x >> 6) * 4 + 1] = w; o[blockIdx.x * 32 + (threadIdx.x >> 6) * 4 + 2] = cu; }
}
int main() {
    unsigned *d; hipMalloc(&d, 64 * 32 * 4); hipMemset(d, 0xff, 64*32*4);
    hipLaunchKernelGGL(k, dim3(64), dim3(512), 0, 0, d);
    unsigned h[64 * 32]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int b = 0; b < 4; ++b) { printf("block %d:", b); for (int w = 0; w < 8; ++w) printf(" w%d(simd %u slot %u cu %u)", w, h[b*32+w*4], h[b*32+w*4+1], h[b*32+w*4+2]); printf("\n"); }
    int cnt[4] = {0,0,0,0}; for (int b = 0; b < 64; ++b) for (int w = 0; w < 8; ++w) cnt[h[b*32+w*4] & 3]++;
    printf("simd histogram %d %d %d %d\n", cnt[0], cnt[1], cnt[2], cnt[3]);
    int bad = 0; for (int b = 0; b < 64; ++b) for (int w = 0; w < 8; ++w) if ((h[b*32+w*4] & 3) != (unsigned)(w & 3)) bad++;
    printf("waves whose simd != wave %% 4: %d of %d\n", bad, 64*8);
}
