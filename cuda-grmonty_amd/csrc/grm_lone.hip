/*
 * grm_lone.hip -- the lone-photon kernels (lone_kernel, early_kernel: the two-wave pipeline of
 * grm_engine.hip §"Lone photons") in a translation unit of their own.
 *
 * Why a second unit of the same source: the pipeline's geometry wave is ONE wave on its SIMD, and a
 * single wave issues one instruction of any kind (VALU, SALU, LDS) per ~4 cycles, so its chain is
 * bound by its instruction count.  grm_engine.hip is built with -disable-machine-licm for the bulk
 * kernel (two waves per SIMD, 256 VGPRs: hoisted constants would cost it spills), which leaves every
 * polynomial and physical constant rematerialised inside the loop -- ~115 s_mov_b32 per geometry
 * step beside ~535 VALU.  Here machine LICM stays on and fma_k is a plain fma: the constants are
 * hoisted into registers once per photon (the lone kernels run one wave per SIMD), the step issues
 * ~100 fewer instructions.  Same operations, same results.
 */
#define GRM_LONE_TU 1
#define GRM_FMA_K_PLAIN 1
#include "grm_engine.hip"

extern "C" hipError_t grm_lone_launch(int which, unsigned grid, hipStream_t s, const void *P, size_t p_size,
                                      const void *C, size_t c_size) {
    if (p_size != sizeof(grm::Params) || c_size != sizeof(Ctl)) return hipErrorInvalidValue; /* built apart */
    grm::Params p;
    Ctl c;
    memcpy(&p, P, sizeof p);
    memcpy(&c, C, sizeof c);
    if (which == 0)
        hipLaunchKernelGGL(lone_kernel, dim3(grid), dim3(128), 0, s, p, c);
    else
        hipLaunchKernelGGL(early_kernel, dim3(1), dim3(64 * 2 * LONE_PAIRS), 0, s, p, c);
    return hipGetLastError();
}
