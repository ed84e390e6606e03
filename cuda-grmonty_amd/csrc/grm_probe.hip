/*
 * grm_probe.hip -- per-function device probes: evaluate one hot-path device function
 * over an array of inputs (one lane per input) so tests can compare every component
 * of the transport step against the CPU oracle.  Not used by the transport path.
 *
 * which  inputs (per item)                          outputs (per item)
 *  0     x[4]                                       g_cov[16]
 *  1     x[4]                                       g^00, g^01
 *  2     x[4]                                       Gamma[4][4][4] (j<=k filled, rest 0)
 *  3     x[4] k[4] dk[4] e_0_s dl                   x[4] k[4] dk[4] e_0_s   (push_photon)
 *  4     x[4]                                       n_e theta_e b u_con u_cov b_con b_cov (19)
 *  5     x[4] k[4]                                  theta nu alpha_scatt alpha_abs (fused), same (separate)
 *  6     w theta_e                                  sigma_hot (lookup)
 *  7     nu n_e theta_e b theta                     j_nu (synch)
 *  8     theta_e                                    K2 (k2_eval)
 *  9     u_con[4] trial[4] x[4]                     e_con[16] e_cov[16]
 * 10     v[4] u[4]                                  vp[4] (boost)
 * 11     seed id ctr0                               8 uniforms
 * 12     k[4] theta_e seed id                       p[4] ctr (sample_electron)
 * 13     k[4] p[4] seed id                          kp[4] ctr (sample_scattered)
 * 14     x[4] k[4]                                  dl (step_size)
 * 15     x[4] k[4]                                  dk[4] (init_dkdlam)
 * 16     w theta_e                                  sigma_hot (numerical quadrature fallback)
 * 17     x                                          e^x K_2(x)
 * 18     seed id dof                                chi^2 sample, ctr
 * 19     x                                          flog(x), ocml log(x)
 * 20     x                                          fsincospi(x) s c, ocml sincospi(x) s c
 * 21     x                                          fexp(x), ocml exp(x)
 * 22     x                                          fexp10(x), ocml exp10(x)
 * 23     x[4] k[4] dk[4] e_0_s dl                   one push attempt: push_attempt x k dk e_1 fail (14), then
 *                                                   push_attempt_quad's (14; four lanes per item, lane q
 *                                                   contracting connection row q -- the lone geometry wave's push)
 */
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "grm_device.h"

using namespace grm;

namespace {

__device__ void store(double *o, int k, double v) { o[k] = v; }

__global__ void probe_kernel(Params P, int which, const double *in, int is, double *out, int os, size_t n) {
    if (which == 23) { /* four lanes per item (the launch has 4 n lanes, quads never straddle an item) */
        const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
        const int q = (int)(threadIdx.x & 3);
        if (t >= n) return;
        const double *a = in + t * is;
        double *o = out + t * os;
        double x[4], k[4], dk[4], xq[4], kq[4], dkq[4];
        for (int i = 0; i < 4; ++i) {
            x[i] = xq[i] = a[i];
            k[i] = kq[i] = a[4 + i];
            dk[i] = dkq[i] = a[8 + i];
        }
        double e1, e1q;
        Trig T;
        Gcov G;
        const bool f = push_attempt(P, x, k, dk, a[12], a[13], e1, T, G);
        const bool fq = push_attempt_quad(P, xq, kq, dkq, a[12], a[13], e1q, T, G, q); /* the lone default */
        if (q == 0) {
            for (int i = 0; i < 4; ++i) {
                store(o, i, x[i]);
                store(o, 4 + i, k[i]);
                store(o, 8 + i, dk[i]);
                store(o, 14 + i, xq[i]);
                store(o, 18 + i, kq[i]);
                store(o, 22 + i, dkq[i]);
            }
            store(o, 12, e1);
            store(o, 13, f ? 1.0 : 0.0);
            store(o, 26, e1q);
            store(o, 27, fq ? 1.0 : 0.0);
        }
        return;
    }
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double *a = in + t * is;
    double *o = out + t * os;
    switch (which) {
    case 0:
    case 1: {
        double x[4] = {a[0], a[1], a[2], a[3]};
        Trig T;
        trig_at(P, x, T);
        Gcov G;
        gcov_from_trig(P, T, G);
        if (which == 0) {
            double g[4][4];
            gcov_full(G, g);
            for (int i = 0; i < 16; ++i) store(o, i, (&g[0][0])[i]);
        } else {
            store(o, 0, G.gn00);
            store(o, 1, G.gn01);
        }
        break;
    }
    case 2: {
        double x[4] = {a[0], a[1], a[2], a[3]};
        Trig T;
        trig_at(P, x, T);
        Conn C;
        connection(P, T, C);
        for (int i = 0; i < 64; ++i) store(o, i, 0.0);
        const int tj[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
        const int tk[10] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};
        for (int i = 0; i < 4; ++i)
            for (int q = 0; q < 10; ++q) store(o, i * 16 + tj[q] * 4 + tk[q], C.c[i][q]);
        break;
    }
    case 3: {
        double x[4], k[4], dk[4];
        for (int i = 0; i < 4; ++i) {
            x[i] = a[i];
            k[i] = a[4 + i];
            dk[i] = a[8 + i];
        }
        double e0s = a[12];
        double bkv[12];
        const Slot bk{bkv, 1};
        push_photon(P, x, k, dk, e0s, a[13], bk);
        for (int i = 0; i < 4; ++i) {
            store(o, i, x[i]);
            store(o, 4 + i, k[i]);
            store(o, 8 + i, dk[i]);
        }
        store(o, 12, e0s);
        break;
    }
    case 4:
    case 5: {
        double x[4] = {a[0], a[1], a[2], a[3]};
        Trig T;
        trig_at(P, x, T);
        Gcov G;
        gcov_from_trig(P, T, G);
        Fluid F;
        fluid_params(P, x, G, F);
        if (which == 4) {
            store(o, 0, F.n_e);
            store(o, 1, F.theta_e);
            store(o, 2, F.b);
            for (int i = 0; i < 4; ++i) {
                store(o, 3 + i, F.u_con[i]);
                store(o, 7 + i, F.u_cov[i]);
                store(o, 11 + i, F.b_con[i]);
                store(o, 15 + i, F.b_cov[i]);
            }
        } else {
            double k[4] = {a[4], a[5], a[6], a[7]};
            const double th = bk_angle(k, F, P.b_unit);
            const double nu = fluid_nu(k, F);
            store(o, 0, th);
            store(o, 1, nu);
            double a_s, a_a; /* the transport kernel's fused evaluation */
            radiation_coeffs(P, k, F, nu, a_s, a_a);
            store(o, 2, a_s);
            store(o, 3, a_a);
            store(o, 4, alpha_inv_scatt(P, nu, F.theta_e, F.n_e)); /* the separate functions */
            store(o, 5, alpha_inv_abs(P, nu, F.theta_e, F.n_e, F.b, th));
        }
        break;
    }
    case 6: store(o, 0, hotcross_lkup(P, a[0], a[1])); break;
    case 7: store(o, 0, synch(P, a[0], a[1], a[2], a[3], a[4])); break;
    case 8: store(o, 0, k2_eval(P, a[0])); break;
    case 9: {
        double u[4] = {a[0], a[1], a[2], a[3]}, tr[4] = {a[4], a[5], a[6], a[7]}, x[4] = {a[8], a[9], a[10], a[11]};
        Trig T;
        trig_at(P, x, T);
        Gcov G;
        gcov_from_trig(P, T, G);
        double ec[4][4];
        make_tetrad(u, tr, G, ec);
        for (int i = 0; i < 4; ++i) {
            double el[4];
            tetrad_cov_row(ec, G, i, el);
            for (int j = 0; j < 4; ++j) {
                store(o, i * 4 + j, ec[i][j]);
                store(o, 16 + i * 4 + j, el[j]);
            }
        }
        break;
    }
    case 10: {
        double v[4] = {a[0], a[1], a[2], a[3]}, u[4] = {a[4], a[5], a[6], a[7]}, vp[4];
        boost(v, u, vp);
        for (int i = 0; i < 4; ++i) store(o, i, vp[i]);
        break;
    }
    case 11: {
        Rng g;
        const uint64_t seed = (uint64_t)a[0];
        g.k0 = (uint32_t)seed;
        g.k1 = (uint32_t)(seed >> 32);
        g.id = (uint64_t)a[1];
        g.ctr = (uint32_t)(uint64_t)a[2];
        g.ctr_hi = (uint32_t)((uint64_t)a[2] >> 32);
        for (int i = 0; i < 8; ++i) store(o, i, uniform(g));
        break;
    }
    case 12:
    case 13:
    case 18: {
        Rng g;
        const int so = which == 12 ? 5 : (which == 13 ? 8 : 0);
        const uint64_t seed = (uint64_t)a[so];
        g.k0 = (uint32_t)seed;
        g.k1 = (uint32_t)(seed >> 32);
        g.id = (uint64_t)a[so + 1];
        g.ctr = 0;
        g.ctr_hi = 0;
        if (which == 12) {
            double k[4] = {a[0], a[1], a[2], a[3]}, p[4];
            sample_electron(g, k, p, a[4]);
            for (int i = 0; i < 4; ++i) store(o, i, p[i]);
            store(o, 4, (double)g.ctr);
        } else if (which == 13) {
            double k[4] = {a[0], a[1], a[2], a[3]}, p[4] = {a[4], a[5], a[6], a[7]}, kp[4];
            sample_scattered(g, k, p, kp);
            for (int i = 0; i < 4; ++i) store(o, i, kp[i]);
            store(o, 4, (double)g.ctr);
        } else {
            store(o, 0, chi_sq(g, (int)a[2]));
            store(o, 1, (double)g.ctr);
        }
        break;
    }
    case 14: {
        double x[4] = {a[0], a[1], a[2], a[3]}, k[4] = {a[4], a[5], a[6], a[7]};
        store(o, 0, step_size(P, x, k));
        break;
    }
    case 15: {
        double x[4] = {a[0], a[1], a[2], a[3]}, k[4] = {a[4], a[5], a[6], a[7]}, dk[4];
        init_dkdlam(P, x, k, dk);
        for (int i = 0; i < 4; ++i) store(o, i, dk[i]);
        break;
    }
    case 16: store(o, 0, hotcross_num(a[0], a[1])); break;
    case 17: store(o, 0, k2_scaled(a[0])); break;
    case 19:
        store(o, 0, flog(a[0]));
        store(o, 1, log(a[0]));
        break;
    case 20: {
        double s0, c0, s1, c1;
        fsincospi(a[0], s0, c0);
        sincospi(a[0], &s1, &c1);
        store(o, 0, s0);
        store(o, 1, c0);
        store(o, 2, s1);
        store(o, 3, c1);
        break;
    }
    case 21:
        store(o, 0, fexp(a[0]));
        store(o, 1, exp(a[0]));
        break;
    case 22:
        store(o, 0, fexp10(a[0]));
        store(o, 1, exp10(a[0]));
        break;
    default: break;
    }
}

} /* namespace */

extern "C" int grm_probe_impl(const Params &P, hipStream_t s, int which, const double *in, int in_stride, double *out,
                              int out_stride, size_t n, std::string &err) {
    if (n == 0) return 0;
    if (!in || !out || in_stride < 1 || out_stride < 1 || which < 0 || which > 23 || (which == 23 && out_stride < 28)) {
        err = "grm_probe: bad arguments";
        return -1;
    }
    double *d_in = nullptr, *d_out = nullptr;
    hipError_t st = hipMalloc(&d_in, n * in_stride * sizeof(double));
    if (st == hipSuccess) st = hipMalloc(&d_out, n * out_stride * sizeof(double));
    if (st == hipSuccess) st = hipMemcpyAsync(d_in, in, n * in_stride * sizeof(double), hipMemcpyHostToDevice, s);
    if (st == hipSuccess) st = hipMemsetAsync(d_out, 0, n * out_stride * sizeof(double), s);
    if (st == hipSuccess) {
        const int B = 64;
        const size_t lanes = which == 23 ? 4 * n : n;
        hipLaunchKernelGGL(probe_kernel, dim3((unsigned)((lanes + B - 1) / B)), dim3(B), 0, s, P, which, d_in, in_stride,
                           d_out, out_stride, n);
        st = hipGetLastError();
    }
    if (st == hipSuccess) st = hipMemcpyAsync(out, d_out, n * out_stride * sizeof(double), hipMemcpyDeviceToHost, s);
    if (st == hipSuccess) st = hipStreamSynchronize(s);
    hipFree(d_in);
    hipFree(d_out);
    if (st != hipSuccess) {
        err = std::string("grm_probe: ") + hipGetErrorString(st);
        return -1;
    }
    return 0;
}
