/*
 * grm_tables.hip -- the model's interpolation tables built on the GPU, the
 * device counterpart of the host builders in host/grm_host.cpp (grm_model_init_device uses it):
 *
 *   hotcross  log10 sigma_hot(w, theta_e), (GRM_HC_N_W+1) x (HC_N_T+1)   hotcross.cpp:60-79, :108-142
 *             (the reference's own GPU builder: hotcross_table.cu:35-65, one thread per entry)
 *   k2        log K_2(1/theta_e), N_E_SAMP+1 points                     jnu_mixed.cpp:57-73
 *   nint, dndlnu_max, NINT+1 points                                     harm_model.cpp:308-338
 *
 * Layout: one workgroup per temperature column of the hotcross table.  The column's electron
 * Lorentz-factor nodes are generated once, sequentially (the same floating-point accumulation as
 * the host loop, so the nodes are the host's nodes), and their Maxwell-Juttner weights and speeds
 * are staged in LDS; each lane then sums one table entry over (mu_e, gamma_e) in the host's order
 * with those weights broadcast from LDS.  K_2 is double precision everywhere: e^x K_2(x) by the
 * trapezoid rule on the integral representation (k2_scaled), not the Abramowitz & Stegun
 * polynomial.  nint: one lane per entry, the sum over frequency in the host's order with exp(weight)
 * and the frequency grid staged in LDS.  Agreement with the host tables is measured in
 * tests/test_gpu_tables.py (std::cyl_bessel_k and glibc vs ocml transcendentals differ in the last
 * bits, so the tables agree to a few ulp rather than bit for bit).
 */
#include <hip/hip_runtime.h>

#include <string>

#include "grm_device.h"

using namespace grm;

namespace {

constexpr int HOT_NODES = 256; /* gamma_e nodes per column: HC_MAX_GAMMA / HC_D_GAMMA_E = 240 */
constexpr int TB = 256;

struct TableConsts {
    double hc_l_min_w, hc_d_l_w, hc_l_min_t, hc_d_l_t;
    double jnu_l_min_t, jnu_d_l_t, jnu_l_min_k, jnu_d_l_k;
    double l_nu_min, d_l_nu, l_b_min, d_l_b, nfac;
};

#define GRM_CR_FN __device__ __forceinline__
#define GRM_CR_LOG(x) log(x)
#include "grm_crlog.h"

/* klein_nishina (hotcross.cpp:144-151), the host expression, each operation rounded as the host's
 * (no contraction) and, below w = 0.1, log(1 + 2w) correctly rounded, as glibc's is: the expression
 * cancels ~6 digits just above w = 1e-3, where ocml's last bit of that log was ~1e-10 of sigma
 * (grm_crlog.h); at w = 0.1 the cancellation makes a last-bit difference ~3e-14 of sigma */
__device__ __forceinline__ double kn_sigma(double w) {
#pragma clang fp contract(off)
    if (w < 1.0e-3) return (1.0 - 2.0 * w);
    const double l = w < 0.1 ? grm_cr::cr_log(1.0 + 2.0 * w) : log(1.0 + 2.0 * w);
    return (3.0 / 4.0) * (2.0 / (w * w) + (1.0 / (2.0 * w) - (1.0 + w) / (w * w * w)) * l +
                          (1.0 + w) / ((1.0 + 2.0 * w) * (1.0 + 2.0 * w)));
}

/* grid[0..HC_N_W] = w, grid[HC_N_W+1..] = theta_e: the host's std::pow values, so that the grid
 * points (and the theta_e < HC_MIN_T switch at the first column) are the host's bit for bit */
__global__ __launch_bounds__(TB) void hot_table_kernel(const double *grid, double *hot) {
#pragma clang fp contract(off) /* every product and sum rounded as the host's (its build has no FMA) */
    __shared__ double s_g[HOT_NODES], s_fw[HOT_NODES], s_v[HOT_NODES];
    __shared__ int s_n;
    const int jj = blockIdx.x;
    const double th = grid[GRM_HC_N_W + 1 + jj];
    if (threadIdx.x == 0) {
        int n = 0;
        for (double g = 1.0 + 0.5 * th * HC_D_GAMMA_E; g < 1.0 + HC_MAX_GAMMA * th && n < HOT_NODES;
             g += th * HC_D_GAMMA_E)
            s_g[n++] = g;
        s_n = n;
    }
    __syncthreads();
    const int n = s_n;
    /* e^x K_2(x) at x = 1 / theta_e, or its small-theta_e asymptote (hotcross.cpp:115-119) */
    const double k2f = th > 1.0e-2 ? k2_scaled(1.0 / th) : sqrt(kPi * th / 2.0);
    for (int t = threadIdx.x; t < n; t += TB) {
        const double g = s_g[t];
        s_fw[t] = 0.5 * ((g * sqrt(g * g - 1.) / (th * k2f)) * exp(-(g - 1.) / th));
        s_v[t] = sqrt(g * g - 1.0) / g;
    }
    __syncthreads();
    for (int ii = threadIdx.x; ii <= GRM_HC_N_W; ii += TB) {
        const double w = grid[ii];
        double sigma;
        if (th < HC_MIN_T && w < HC_MIN_W) {
            sigma = SIGMA_THOMSON;
        } else if (th < HC_MIN_T) {
            sigma = kn_sigma(w) * SIGMA_THOMSON;
        } else {
            double cross = 0.0;
            for (double mu = -1.0 + 0.5 * HC_D_MU_E; mu < 1.0; mu += HC_D_MU_E)
                for (int t = 0; t < n; ++t) {
                    const double f = 1.0 - mu * s_v[t];
                    cross += th * HC_D_MU_E * HC_D_GAMMA_E * (kn_sigma(w * s_g[t] * f) * f) * s_fw[t];
                }
            sigma = cross * SIGMA_THOMSON;
        }
        hot[(size_t)ii * (HC_N_T + 1) + jj] = grm_cr::grm_log10(sigma); /* glibc's log10 construction */
    }
}

__global__ __launch_bounds__(TB) void k2_table_kernel(TableConsts K, double *k2) {
    const int q = blockIdx.x * TB + threadIdx.x;
    if (q > GRM_N_E_SAMP) return;
    const double x = 1.0 / exp(q * K.jnu_d_l_t + K.jnu_l_min_t);
    k2[q] = log(k2_scaled(x)) - x; /* log K_2(x) = log(e^x K_2(x)) - x */
}

/* F(K) of jnu_mixed.cpp:113-125 at theta_e = 1 from the host-built ftab */
__device__ __forceinline__ double f_eval1(const TableConsts &K, const double *ftab, double b_mag, double nu) {
    const double k = (9.0 * kPi * ME * CL / EE) * nu / (b_mag * 1.0 * 1.0);
    if (k > 1.0e7) return 0.0;
    if (k < 0.002) {
        const double x = pow(k, 1.0 / 3.0);
        return x * (37.67503800178 + 2.240274341836 * x);
    }
    double d = (log(k) - K.jnu_l_min_k) / K.jnu_d_l_k;
    const int i = min((int)d, GRM_N_E_SAMP - 1);
    d -= i;
    return exp((1.0 - d) * ftab[i] + d * ftab[i + 1]);
}

__global__ __launch_bounds__(TB) void nint_table_kernel(TableConsts K, const double *ftab, const double *weight,
                                                         double *nint, double *dmax_out) {
    __shared__ double s_nu[GRM_N_E_SAMP], s_ew[GRM_N_E_SAMP];
    for (int q = threadIdx.x; q < GRM_N_E_SAMP; q += TB) {
        s_nu[q] = exp(q * K.d_l_nu + K.l_nu_min);
        s_ew[q] = exp(weight[q]) + 1.0e-100;
    }
    __syncthreads();
    const int i = blockIdx.x * TB + threadIdx.x;
    if (i > GRM_NINT) return;
    const double b_mag = exp(i * K.d_l_b + K.l_b_min);
    double s = 0.0, dmax = 0.0;
    for (int q = 0; q < GRM_N_E_SAMP; ++q) {
        const double dn = f_eval1(K, ftab, b_mag, s_nu[q]) / s_ew[q];
        if (dn > dmax) dmax = dn;
        s += K.d_l_nu * dn;
    }
    s *= K.nfac;
    nint[i] = log(s);
    dmax_out[i] = log(dmax);
}

bool chk(hipError_t st, const char *what, std::string &err) {
    if (st == hipSuccess) return true;
    err = std::string(what) + ": " + hipGetErrorString(st);
    return false;
}

} /* namespace */

/* library-internal (host/grm_host.cpp, C linkage there): c[] = the TableConsts fields in order */
extern "C" int grm_tables_hot_k2_device(int device, const double c[13], const double *grid, double *hot, double *k2, float *ms,
                                        std::string &err) {
    TableConsts K;
    static_assert(sizeof(TableConsts) == 13 * sizeof(double), "TableConsts layout");
    __builtin_memcpy(&K, c, sizeof(K));
    const size_t n_hot = (size_t)(GRM_HC_N_W + 1) * (HC_N_T + 1), n_k2 = GRM_N_E_SAMP + 1;
    const size_t n_grid = (size_t)GRM_HC_N_W + 1 + HC_N_T + 1;
    double *d_hot = nullptr, *d_k2 = nullptr, *d_grid = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool ok = chk(hipSetDevice(device), "hipSetDevice", err) && chk(hipMalloc(&d_hot, n_hot * sizeof(double)), "hot", err) &&
              chk(hipMalloc(&d_k2, n_k2 * sizeof(double)), "k2", err) &&
              chk(hipMalloc(&d_grid, n_grid * sizeof(double)), "grid", err) &&
              chk(hipMemcpy(d_grid, grid, n_grid * sizeof(double), hipMemcpyHostToDevice), "H2D", err) &&
              chk(hipEventCreate(&e0), "event", err) && chk(hipEventCreate(&e1), "event", err) &&
              chk(hipEventRecord(e0, 0), "event", err);
    if (ok) {
        hipLaunchKernelGGL(hot_table_kernel, dim3(HC_N_T + 1), dim3(TB), 0, 0, d_grid, d_hot);
        hipLaunchKernelGGL(k2_table_kernel, dim3((unsigned)((n_k2 + TB - 1) / TB)), dim3(TB), 0, 0, K, d_k2);
        ok = chk(hipGetLastError(), "table kernels", err) && chk(hipEventRecord(e1, 0), "event", err) &&
             chk(hipEventSynchronize(e1), "table kernels", err) && chk(hipEventElapsedTime(ms, e0, e1), "event", err) &&
             chk(hipMemcpy(hot, d_hot, n_hot * sizeof(double), hipMemcpyDeviceToHost), "D2H", err) &&
             chk(hipMemcpy(k2, d_k2, n_k2 * sizeof(double), hipMemcpyDeviceToHost), "D2H", err);
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d_hot);
    (void)hipFree(d_k2);
    (void)hipFree(d_grid);
    return ok ? 0 : -1;
}

extern "C" int grm_tables_nint_device(int device, const double c[13], const double *ftab, const double *weight, double *nint,
                           double *dndlnu_max, float *ms, std::string &err) {
    TableConsts K;
    __builtin_memcpy(&K, c, sizeof(K));
    const size_t n_t = GRM_N_E_SAMP + 1, n_i = GRM_NINT + 1;
    double *d_f = nullptr, *d_w = nullptr, *d_n = nullptr, *d_m = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool ok = chk(hipSetDevice(device), "hipSetDevice", err) && chk(hipMalloc(&d_f, n_t * sizeof(double)), "ftab", err) &&
              chk(hipMalloc(&d_w, n_t * sizeof(double)), "weight", err) &&
              chk(hipMalloc(&d_n, n_i * sizeof(double)), "nint", err) &&
              chk(hipMalloc(&d_m, n_i * sizeof(double)), "dndlnu_max", err) &&
              chk(hipMemcpy(d_f, ftab, n_t * sizeof(double), hipMemcpyHostToDevice), "H2D", err) &&
              chk(hipMemcpy(d_w, weight, n_t * sizeof(double), hipMemcpyHostToDevice), "H2D", err) &&
              chk(hipEventCreate(&e0), "event", err) && chk(hipEventCreate(&e1), "event", err) &&
              chk(hipEventRecord(e0, 0), "event", err);
    if (ok) {
        hipLaunchKernelGGL(nint_table_kernel, dim3((unsigned)((n_i + TB - 1) / TB)), dim3(TB), 0, 0, K, d_f, d_w, d_n, d_m);
        ok = chk(hipGetLastError(), "nint kernel", err) && chk(hipEventRecord(e1, 0), "event", err) &&
             chk(hipEventSynchronize(e1), "nint kernel", err) && chk(hipEventElapsedTime(ms, e0, e1), "event", err) &&
             chk(hipMemcpy(nint, d_n, n_i * sizeof(double), hipMemcpyDeviceToHost), "D2H", err) &&
             chk(hipMemcpy(dndlnu_max, d_m, n_i * sizeof(double), hipMemcpyDeviceToHost), "D2H", err);
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d_f);
    (void)hipFree(d_w);
    (void)hipFree(d_n);
    (void)hipFree(d_m);
    return ok ? 0 : -1;
}
