/* Single-wave latency of the geodesic push pieces (the lone-photon geometry wave's critical path):
 * one wave, a serially dependent chain of N evaluations, cycles per evaluation by s_memtime.
 * Build: hipcc --offload-arch=gfx950 -O3 -I../../cuda-grmonty_amd/csrc push_lat.hip -o push_lat */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "grm_device.h"
using namespace grm;

template <int WHAT>
__global__ __launch_bounds__(64) void lat_kernel(Params P, const double *s, double *o, unsigned long long *cyc, int n) {
    double x0[4], k0[4], dk0[4];
    for (int i = 0; i < 4; ++i) { x0[i] = s[i]; k0[i] = s[4 + i]; dk0[i] = s[8 + i]; }
    const double e0 = s[12], dl = s[13];
    double dep = 0.0, acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < n; ++it) {
        double x[4], k[4], dk[4];
        for (int i = 0; i < 4; ++i) { x[i] = x0[i] + dep; k[i] = k0[i]; dk[i] = dk0[i]; }
        double r;
        if (WHAT == 0) { Trig T; trig_at(P, x, T); r = T.r1 + T.sth + T.cth; }
        else if (WHAT == 1) { Trig T; trig_at(P, x, T); Conn C; connection(P, T, C); r = C.c[0][0] + C.c[3][9] + C.c[2][6]; }
        else if (WHAT == 2) { double e1; Trig T; Gcov G; bool f = push_attempt(P, x, k, dk, e0, dl, e1, T, G); r = e1 + k[0] + x[1] + dk[2] + (f ? 1.0 : 0.0); }
        else { r = step_size(P, x, k); }
        acc += r;
        dep = r * 0.0;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o[WHAT] = acc; cyc[WHAT] = t1 - t0; cyc[4 + WHAT] = r1 - r0; }
}

int main() {
    Params P{};
    P.a = 0.9375; P.h_slope = 0.3; P.r0 = 0.0; P.xs1 = 0.3; P.xe2 = 1.0;
    /* a photon near r = 6 M off the pole: x, k (k^0 from the null condition approx), dk/dlambda */
    double h[14] = {0.0, 1.79, 0.21, 0.4, 1.0, 0.12, 0.03, 0.05, 0.0, 0.0, 0.0, 0.0, -0.9, 0.01};
    double *s, *o; unsigned long long *cyc;
    hipMalloc(&s, sizeof h); hipMalloc(&o, 8 * 8); hipMalloc(&cyc, 8 * 8);
    /* dk from the connection at x, as the transport does */
    hipMemcpy(s, h, sizeof h, hipMemcpyHostToDevice);
    const int n = 20000;
    unsigned long long c[8] = {0};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(lat_kernel<0>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<1>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<2>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<3>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipDeviceSynchronize();
    }
    hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
    const char *nm[4] = {"trig_at", "trig+connection", "push_attempt", "step_size"};
    for (int w = 0; w < 4; ++w) printf("%-16s %8.1f cycles (s_memtime) %8.1f ns per evaluation, one wave\n", nm[w], (double)c[w] / n, c[4 + w] * 10.0 / n);
    return 0;
}
