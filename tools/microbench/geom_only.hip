/* Rate of the lone pipeline's geometry wave (lone_geometry, the engine's own code) with a trivial
 * consumer instead of the interaction wave: does the geometry wave's chain run at the single-wave
 * push rate (push_lat.hip), and what does a busy neighbour wave with a large code footprint cost it?
 * Build: hipcc --offload-arch=gfx950 -O3 -mllvm -disable-machine-licm -I../../cuda-grmonty_amd/csrc
 *        geom_only.hip -o geom_only -L/opt/rocm/lib -lrccl -L../../cuda-grmonty_amd -lgrmonty_amd
 *        (includes the engine translation unit; the library supplies emission / probe symbols) */
#include "../../cuda-grmonty_amd/csrc/grm_engine.hip"
#include <cstdlib>

namespace {
/* MODE 0: the consumer only advances cons.  MODE 1: between polls it runs Compton sampling, a log
 * and an exp (a different instruction stream on the other SIMD; registers only). */
template <int MODE>
__global__ __launch_bounds__(128) void geo_kernel(Params P, Ctl C, const double *st, unsigned long long *out, int n) {
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    LonePair &pr = s_pair[0];
    if (threadIdx.x < LONE_RING) pr.ring[threadIdx.x].tag = 0;
    if (threadIdx.x == 0) { pr.ctl.cons = 0; pr.ctl.req = 0; }
    __syncthreads();
    if (wave == 1) { lone_geometry(P, C, lane, pr); return; }
    if (lane == 0) {
        double x[4], k[4], dk[4];
        for (int i = 0; i < 4; ++i) { x[i] = st[i]; k[i] = st[4 + i]; }
        init_dkdlam(P, x, k, dk);
        Trig T; trig_at(P, x, T); Gcov G; gcov_from_trig(P, T, G);
        pack13(pr.ctl.rs, x, k, dk, -(k[0] * G.g00 + k[1] * G.g01 + k[3] * G.g03));
        __hip_atomic_store(&pr.ctl.req, 1ull << 32, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    Rng g; g.k0 = 1; g.k1 = 2; g.id = lane; g.ctr = 0; g.ctr_hi = 0;
    double acc = 0.0, kk[4] = {1.0, 0.3, 0.2, 0.1}, p[4], kp[4];
    unsigned long long t0 = 0;
    for (int si = 0; si < n; ++si) {
        const unsigned long long want = (1ull << 32) | (unsigned long long)(si + 1);
        while (__hip_atomic_load(&pr.ring[si % LONE_RING].tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != want) {
            if (MODE == 1) {
                /* register-only work (no table or zone loads: P has no device tables here) */
                sample_scattered(g, kk, p, kp);
                acc += kp[0] + flog(1.0 + fabs(kp[1])) + fexp(-fabs(kp[2]));
            } else {
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (si == 1000) t0 = __builtin_amdgcn_s_memtime();
        if (lane == 0) __hip_atomic_store(&pr.ctl.cons, (unsigned long long)(si + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        __hip_atomic_store(&pr.ctl.req, LONE_STOP, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        out[MODE] = t1 - t0;
        out[4 + MODE] = __double_as_longlong(acc);
    }
}
}  // namespace

int main() {
    Params P{};
    P.a = 0.9375; P.h_slope = 0.3; P.r0 = 0.0; P.xs1 = 0.3; P.xe2 = 1.0; P.x1_min = 0.3; P.x1_max = 3.7;
    params_metric(P);
    double h[8] = {0.0, 2.2, 0.45, 0.0, 1.0, 0.0, 0.0, 0.3};
    if (getenv("GEO_STATE")) sscanf(getenv("GEO_STATE"), "%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf", h, h + 1, h + 2, h + 3, h + 4, h + 5, h + 6, h + 7);
    double *st; unsigned long long *out;
    (void)hipMalloc(&st, sizeof h); (void)hipMalloc(&out, 64); (void)hipMemset(out, 0, 64);
    (void)hipMemcpy(st, h, sizeof h, hipMemcpyHostToDevice);
    Ctl C{};
    const int n = 21000;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(geo_kernel<0>, dim3(1), dim3(128), 0, 0, P, C, st, out, n);
        hipLaunchKernelGGL(geo_kernel<1>, dim3(1), dim3(128), 0, 0, P, C, st, out, n);
        const hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess || hipGetLastError() != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(e)); return 1; }
    }
    unsigned long long o[8];
    (void)hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
    printf("geometry wave, trivial consumer:      %.1f cycles/step (s_memtime)\n", (double)o[0] / (n - 1001));
    printf("geometry wave, busy neighbour wave:   %.1f cycles/step\n", (double)o[1] / (n - 1001));
    return 0;
}
