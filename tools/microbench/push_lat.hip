/* Single-wave latency of the geodesic push pieces (the lone-photon geometry wave's critical path):
 * one wave, a serially dependent chain of N evaluations, cycles per evaluation by s_memtime.
 * Build: hipcc --offload-arch=gfx950 -O3 -I../../cuda-grmonty_amd/csrc push_lat.hip -o push_lat */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "grm_device.h"
using namespace grm;

/* push_finish with the second corrector pass computed unconditionally and selected (no branch on
 * the first pass's error; MAX_ITER = 2) */
__device__ __forceinline__ bool push_finish_spec(const Conn &C, double k[4], double kp[4], double dk[4], double dl,
                                                 double e_0_s, double g00, double g01, double g03, double &e_1) {
    const double dl_2 = 0.5 * dl;
    double kc[4] = {kp[0], kp[1], kp[2], kp[3]};
    double dk1[4], kp1[4], dk2[4], kp2[4];
    double err1 = 0.0, err2 = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        dk1[i] = geo_rhs(C, i, kc);
        kp1[i] = k[i] + dl_2 * dk1[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        dk2[i] = geo_rhs(C, i, kp1);
        kp2[i] = k[i] + dl_2 * dk2[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) err1 += fratio_tol(kc[i] - kp1[i], kp1[i] + EPS);
#pragma unroll
    for (int i = 0; i < 4; ++i) err2 += fratio_tol(kp1[i] - kp2[i], kp2[i] + EPS);
    const bool two = err1 > E_TOL;
    const double err = two ? err2 : err1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        k[i] = two ? kp2[i] : kp1[i];
        dk[i] = two ? dk2[i] : dk1[i];
    }
    e_1 = -(k[0] * g00 + k[1] * g01 + k[3] * g03);
    const bool err_e = fabs(e_1 - e_0_s) > 1.0e-4 * fabs(e_0_s);
    return (err_e || err > E_TOL || isnan(err) || isinf(err));
}

__device__ __forceinline__ double tree40(const Conn &C) {
    double t[40];
    for (int i = 0; i < 40; ++i) t[i] = (&C.c[0][0])[i];
    for (int w = 1; w < 40; w *= 2)
        for (int i = 0; i + w < 40; i += 2 * w) t[i] += t[i + w];
    return t[0];
}

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
        else if (WHAT == 3) { r = step_size(P, x, k); }
        else if (WHAT == 4) { Trig T; trig_at(P, x, T); Conn C; connection(P, T, C); r = tree40(C); }
        else if (WHAT == 5) { /* kick + trig + connection + metric, no corrector */
            double kp[4]; push_kick(x, k, dk, dl, kp); Trig T; trig_at(P, x, T); Conn C; connection(P, T, C);
            Gcov G; gcov_from_trig(P, T, G); r = tree40(C) + G.g00 + G.g01 + G.g03 + kp[0] + kp[1] + kp[2] + kp[3]; }
        else if (WHAT == 6) { /* push_attempt with the speculative second corrector pass */
            double kp[4]; push_kick(x, k, dk, dl, kp); Trig T; trig_at(P, x, T); Conn C; connection(P, T, C);
            Gcov G; gcov_from_trig(P, T, G); double e1;
            bool f = push_finish_spec(C, k, kp, dk, dl, e0, G.g00, G.g01, G.g03, e1);
            r = e1 + k[0] + x[1] + dk[2] + (f ? 1.0 : 0.0); }
        else if (WHAT == 8) { /* quad-parallel push (push_attempt_quad) */
            double e1; Trig T; Gcov G; bool f = push_attempt_quad(P, x, k, dk, e0, dl, e1, T, G, threadIdx.x & 3);
            r = e1 + k[0] + x[1] + dk[2] + (f ? 1.0 : 0.0); }
        else if (WHAT == 9) { /* kick + trig + quad rows (divergent blocks) + metric, no corrector */
            double kp[4]; push_kick(x, k, dk, dl, kp); Trig T; trig_at(P, x, T); double L[10];
            connection_quad_row(P, T, threadIdx.x & 3, L); Gcov G; gcov_from_trig(P, T, G);
            r = L[0] + L[1] + L[2] + L[3] + L[4] + L[5] + L[6] + L[7] + L[8] + L[9] + G.g00 + G.g01 + G.g03 + kp[0] + kp[1] + kp[2] + kp[3]; }
        else if (WHAT == 10) { /* kick + trig + quad rows (selected) + metric, no corrector */
            double kp[4]; push_kick(x, k, dk, dl, kp); Trig T; trig_at(P, x, T); double L[10];
            connection_quad_sel(P, T, threadIdx.x & 3, L); Gcov G; gcov_from_trig(P, T, G);
            r = L[0] + L[1] + L[2] + L[3] + L[4] + L[5] + L[6] + L[7] + L[8] + L[9] + G.g00 + G.g01 + G.g03 + kp[0] + kp[1] + kp[2] + kp[3]; }
        else if (WHAT == 11) { /* quad push, selected rows */
            double e1; Trig T; Gcov G; bool f = push_attempt_quad<1>(P, x, k, dk, e0, dl, e1, T, G, threadIdx.x & 3);
            r = e1 + k[0] + x[1] + dk[2] + (f ? 1.0 : 0.0); }
        else if (WHAT == 12) { /* kick + trig + 40 rows + metric summed like 9/10 */
            double kp[4]; push_kick(x, k, dk, dl, kp); Trig T; trig_at(P, x, T); Conn C; connection(P, T, C);
            Gcov G; gcov_from_trig(P, T, G); double a = 0.0; for (int i = 0; i < 4; ++i) for (int j = 0; j < 10; ++j) a += C.c[i][j];
            r = a + G.g00 + G.g01 + G.g03 + kp[0] + kp[1] + kp[2] + kp[3]; }
        else { /* corrector iteration count of the state: 1 or 2 */
            double e1; Trig T; Gcov G; double kp[4]; push_kick(x, k, dk, dl, kp); trig_at(P, x, T); Conn C; connection(P, T, C);
            double kc[4] = {kp[0], kp[1], kp[2], kp[3]}, err = 0.0;
            for (int i = 0; i < 4; ++i) { double d = geo_rhs(C, i, kc); double kq = k[i] + 0.5 * dl * d; err += fabs((kc[i] - kq) / (kq + EPS)); }
            r = err > E_TOL ? 2.0 : 1.0; (void)e1; (void)G; }
        acc += r;
        dep = r * 0.0;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o[WHAT] = acc; cyc[WHAT] = t1 - t0; cyc[20 + WHAT] = r1 - r0; }
}

/* push_attempt vs push_attempt_quad on lane-varied states (lane >> 2 picks dl): every output bit */
template <int SEL>
__global__ __launch_bounds__(64) void quad_check(Params P, const double *s, double *o) {
    double x[4], k[4], dk[4], xq[4], kq[4], dkq[4];
    for (int i = 0; i < 4; ++i) { x[i] = xq[i] = s[i]; k[i] = kq[i] = s[4 + i]; }
    init_dkdlam(P, x, k, dk);
    for (int i = 0; i < 4; ++i) dkq[i] = dk[i];
    double e0;
    { Trig T0; trig_at(P, x, T0); Gcov G0; gcov_from_trig(P, T0, G0); e0 = -(k[0] * G0.g00 + k[1] * G0.g01 + k[3] * G0.g03); }
    const double dl = s[13] * (double)(1 << (threadIdx.x >> 2)) * 0.037;
    double e1, e1q; Trig T; Gcov G;
    const bool f = push_attempt(P, x, k, dk, e0, dl, e1, T, G);
    const bool fq = SEL ? push_attempt_quad<1>(P, xq, kq, dkq, e0, dl, e1q, T, G, threadIdx.x & 3)
                        : push_attempt_quad<0>(P, xq, kq, dkq, e0, dl, e1q, T, G, threadIdx.x & 3);
    double *d = o + 32 * threadIdx.x;
    for (int i = 0; i < 4; ++i) { d[i] = x[i]; d[4 + i] = k[i]; d[8 + i] = dk[i]; d[16 + i] = xq[i]; d[20 + i] = kq[i]; d[24 + i] = dkq[i]; }
    d[12] = e1; d[13] = f; d[28] = e1q; d[29] = fq;
}

/* wave 0 chains pushes as above while the other waves of the workgroup run the same chain (busy
 * neighbours): does a second wave of the workgroup share wave 0's SIMD? */
__global__ __launch_bounds__(256) void pair_kernel(Params P, const double *s, double *o, unsigned long long *cyc, int n) {
    const int wave = threadIdx.x >> 6;
    double x0[4], k0[4], dk0[4];
    for (int i = 0; i < 4; ++i) { x0[i] = s[i]; k0[i] = s[4 + i]; dk0[i] = s[8 + i]; }
    const double e0 = s[12], dl = s[13];
    double dep = 0.0, acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        double x[4], k[4], dk[4];
        for (int i = 0; i < 4; ++i) { x[i] = x0[i] + dep; k[i] = k0[i]; dk[i] = dk0[i]; }
        double e1; Trig T; Gcov G; bool f = push_attempt(P, x, k, dk, e0, dl, e1, T, G);
        const double r = e1 + k[0] + x[1] + dk[2] + (f ? 1.0 : 0.0);
        acc += r;
        dep = r * 0.0;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if ((threadIdx.x & 63) == 0) { o[16 + wave] = acc; cyc[16 + wave] = t1 - t0; cyc[24 + wave] = hw; }
}

/* wave 0 chains pushes; the other waves run different heavy code (Compton scattering samples):
 * does foreign code on the other SIMDs of the CU slow the chain (instruction cache, arbitration)? */
__global__ __launch_bounds__(256) void foreign_kernel(Params P, const double *s, double *o, unsigned long long *cyc, int n,
                                                      int busy) {
    const int wave = threadIdx.x >> 6;
    if (wave == 0) {
        double x0[4], k0[4], dk0[4];
        for (int i = 0; i < 4; ++i) { x0[i] = s[i]; k0[i] = s[4 + i]; dk0[i] = s[8 + i]; }
        const double e0 = s[12], dl = s[13];
        double dep = 0.0, acc = 0.0;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int it = 0; it < n; ++it) {
            double x[4], k[4], dk[4];
            for (int i = 0; i < 4; ++i) { x[i] = x0[i] + dep; k[i] = k0[i]; dk[i] = dk0[i]; }
            double e1; Trig T; Gcov G; bool f = push_attempt(P, x, k, dk, e0, dl, e1, T, G);
            const double r = e1 + k[0] + x[1] + dk[2] + (f ? 1.0 : 0.0);
            acc += r;
            dep = r * 0.0;
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0) { o[28] = acc; cyc[28] = t1 - t0; }
        if (threadIdx.x == 0) __hip_atomic_store(cyc + 29, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else if (busy) {
        Rng g; g.k0 = 1; g.k1 = 2; g.id = threadIdx.x; g.ctr = 0; g.ctr_hi = 0;
        double acc = 0.0;
        double k[4] = {1.0, 0.3, 0.2, 0.1}, p[4], kp[4];
        while (__hip_atomic_load(cyc + 29, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            sample_scattered(g, k, p, kp);
            acc += kp[0] + kp[1] + p[2];
            k[1] = 0.3 + acc * 1e-300;
        }
        if ((threadIdx.x & 63) == 0) o[29 + wave] = acc;
    }
}

int main() {
    Params P{};
    P.a = 0.9375; P.h_slope = 0.3; P.r0 = 0.0; P.xs1 = 0.3; P.xe2 = 1.0;
    params_metric(P);
    /* a photon near r = 6 M off the pole: x, k (k^0 from the null condition approx), dk/dlambda */
    double h[14] = {0.0, 1.79, 0.21, 0.4, 1.0, 0.12, 0.03, 0.05, 0.0, 0.0, 0.0, 0.0, -0.9, 0.01};
    if (getenv("PL_STATE")) sscanf(getenv("PL_STATE"), "%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf", h, h+1, h+2, h+3, h+4, h+5, h+6, h+7, h+8, h+9, h+10, h+11, h+12, h+13);
    double *s, *o; unsigned long long *cyc;
    hipMalloc(&s, sizeof h); hipMalloc(&o, 40 * 8); hipMalloc(&cyc, 40 * 8);
    /* dk from the connection at x, as the transport does */
    hipMemcpy(s, h, sizeof h, hipMemcpyHostToDevice);
    const int n = 20000;
    unsigned long long c[40] = {0};
    static_assert(40 >= 18, "cycle slots");
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(lat_kernel<0>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<1>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<2>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<3>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<4>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<5>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<6>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<7>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<8>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<9>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<10>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<11>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipLaunchKernelGGL(lat_kernel<12>, dim3(1), dim3(64), 0, 0, P, s, o, cyc, n);
        hipDeviceSynchronize();
    }
    hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
    const char *nm[13] = {"trig_at", "trig+conn(3 used)", "push_attempt", "step_size", "trig+conn(40)", "kick..metric",
                         "push_spec2", "iterations", "push_attempt_quad", "kick..metric quadrow", "kick..metric quadsel",
                         "push_quad_sel", "kick..metric 40sum"};
    double oh[16];
    hipMemcpy(oh, o, sizeof oh, hipMemcpyDeviceToHost);
    for (int w = 0; w < 13; ++w) if (w != 7) printf("%-18s %8.1f cycles (s_memtime) %8.1f ns per evaluation, one wave\n", nm[w], (double)c[w] / n, c[20 + w] * 10.0 / n);
    printf("corrector passes of the test state: %.0f\n", oh[7] / n);
    {
        double *oc; hipMalloc(&oc, 64 * 32 * 8);
        for (int sel = 0; sel < 2; ++sel) {
        if (sel) hipLaunchKernelGGL(quad_check<1>, dim3(1), dim3(64), 0, 0, P, s, oc);
        else hipLaunchKernelGGL(quad_check<0>, dim3(1), dim3(64), 0, 0, P, s, oc);
        double hc[64 * 32]; hipMemcpy(hc, oc, sizeof hc, hipMemcpyDeviceToHost);
        int bad = 0, fails = 0, nans = 0;
        for (int l = 0; l < 64; ++l) {
            const double *d = hc + 32 * l;
            for (int i = 0; i < 13; ++i) {
                const int w = i < 12 ? i : 12, wq = i < 12 ? 16 + i : 28;
                const bool same = memcmp(d + w, d + wq, 8) == 0 || (d[w] != d[w] && d[wq] != d[wq]);
                nans += d[w] != d[w];
                if (!same && bad++ < 4) printf("  lane %d word %d: %.17g vs %.17g\n", l, i, d[w], d[wq]);
            }
            bad += d[13] != d[29]; fails += d[13] != 0.0;
        }
        printf("quad check (%s rows): %d differing words over 64 lanes (16 step lengths, %d failing attempts, %d NaN words)\n",
               sel ? "selected" : "divergent", bad, fails, nans);
        }
        hipFree(oc);
    }
    for (int nw = 1; nw <= 4; ++nw) {
        hipLaunchKernelGGL(pair_kernel, dim3(1), dim3(64 * nw), 0, 0, P, s, o, cyc, n);
        hipDeviceSynchronize();
        hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
        printf("workgroup of %d waves: cycles per push", nw);
        for (int w = 0; w < nw; ++w) printf("  w%d %.1f (SIMD %llu)", w, (double)c[16 + w] / n, (c[24 + w] >> 4) & 3);
        printf("\n");
    }
    for (int busy = 0; busy <= 1; ++busy) {
        hipMemset(cyc, 0, 40 * 8);
        hipLaunchKernelGGL(foreign_kernel, dim3(1), dim3(256), 0, 0, P, s, o, cyc, n, busy);
        hipDeviceSynchronize();
        hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
        printf("push chain with %s on the other 3 waves: %.1f cycles per push\n", busy ? "Compton sampling" : "nothing",
               (double)c[28] / n);
    }
    return 0;
}
