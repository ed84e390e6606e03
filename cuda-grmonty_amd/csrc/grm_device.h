/*
 * grm_device.h -- device-side physics of the transport hot path (HIP, gfx950).
 *
 * Same algorithm as the reference CPU path (m-torhan/cuda-grmonty, CPU semantics
 * chosen over its CUDA port where they differ -- SURVEY.md §8 quirks Q1-Q8),
 * written for CDNA4: all state in VGPRs, no 4x4 heap temporaries, shared trig
 * between the metric and the connection at one point, iterative (stackless)
 * geodesic sub-stepping, fp64 throughout.
 *
 * Included only by the .hip translation units of this package.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/grmonty_amd.h"
#include "../../include/grmonty_amd_debug.h"

namespace grm {

/* ---- constants: reference consts.hpp:14-157 (same literals) ---- */
constexpr double kPi = 3.141592653589793238462643383279502884;
constexpr double kLog10E = 0.43429448190325182765112891891660508; /* 1 / ln 10 */
constexpr double kSqrt2 = 1.414213562373095048801688724209698079;
constexpr double EPS = 1.0e-40;
constexpr double THETA_E_MIN = 0.3, TP_OVER_TE = 3.0;
constexpr double WEIGHT_MIN = 1.0e31, ROULETTE = 1.0e4;
constexpr double STEP_EPS = 0.04, E_TOL = 1.0e-3;
constexpr int MAX_ITER = 2, MAX_N_STEP = 1280000, MAX_SUBDIV = 7;
constexpr double EE = 4.80320680e-10, CL = 2.99792458e10, ME = 9.1093826e-28, MP = 1.67262171e-24;
constexpr double HPL = 6.6260693e-27;
constexpr double SIGMA_THOMSON = 0.665245873e-24;
constexpr double HC_MIN_W = 1.0e-12, HC_MAX_W = 1.0e6, HC_MIN_T = 1.0e-4, HC_MAX_T = 1.0e4;
constexpr int HC_N_T = 80;
constexpr double HC_MAX_GAMMA = 12.0, HC_D_MU_E = 0.05, HC_D_GAMMA_E = 0.05;
constexpr double JNU_MAX_T = 1.0e2, JNU_CST = 1.88774862536;
constexpr double SPEC_D_L_E = 0.25;
constexpr int N_TH_BINS = GRM_N_TH_BINS, N_E_BINS = GRM_N_E_BINS;

/* ---- division ----
 * An IEEE fp64 divide is 11 VALU ops on CDNA (div_scale x2, rcp, 5 fma, mul, div_fmas, div_fixup).
 * The transport step's divisors are finite, normal, non-zero physical quantities, so the hot path
 * divides with v_rcp_f64 + two Newton steps + one residual correction (7 ops, <= 1 ulp from the
 * correctly rounded quotient -- below the fp-contraction differences the CPU reference already has
 * from one compiler to another). */
__device__ __forceinline__ double frcp(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    e = fma(-b, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ double fdiv(double a, double b) {
    const double r = frcp(b);
    const double q = a * r;
    return fma(fma(-b, q, a), r, q);
}
/* |a| / |b| for a tolerance test only (one Newton step, ~1e-16 relative) */
__device__ __forceinline__ double fratio_tol(double a, double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(r, fma(-b, r, 1.0), r);
    return fabs(a * r);
}
/* ---- polynomial coefficients from SGPRs ----
 * d = a b + c for a compile-time constant c.  Left to itself the compiler evaluates a Horner step
 * as v_fmac (d = c tied to the destination) and so first copies c into a VGPR pair: two v_mov_b32
 * per coefficient per evaluation inside the persistent loop (machine LICM is off, see the Makefile),
 * i.e. three VALU instructions per step of every polynomial.  With c as an SGPR operand of
 * v_fma_f64 the copy is two s_mov_b32 on the scalar unit: one VALU instruction.  Same operation,
 * same rounding. */
__device__ __forceinline__ double fma_k(double a, double b, double c) {
#ifdef GRM_FMA_K_PLAIN
    return fma(a, b, c);
#endif
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}
#define GRM_K(h) __builtin_bit_cast(double, (unsigned long long)(h))

/* ocml's exp and exp10 (the same operations in the same order, so bit-identical results,
 * tests/test_gpu_probes.py) with their coefficients through fma_k: k = rint(x log2 e), a two-part
 * ln 2 reduction, a degree-11 minimax polynomial, ldexp; x > 1024 gives inf, x < -1075 zero. */
__device__ __forceinline__ double exp_poly(double r) {
    double p = fma_k(r, GRM_K(0x3e5ade156a5dcb37ull), GRM_K(0x3e928af3fca7ab0cull));
    p = fma_k(r, p, GRM_K(0x3ec71dee623fde64ull));
    p = fma_k(r, p, GRM_K(0x3efa01997c89e6b0ull));
    p = fma_k(r, p, GRM_K(0x3f2a01a014761f6eull));
    p = fma_k(r, p, GRM_K(0x3f56c16c1852b7b0ull));
    p = fma_k(r, p, GRM_K(0x3f81111111122322ull));
    p = fma_k(r, p, GRM_K(0x3fa55555555502a1ull));
    p = fma_k(r, p, GRM_K(0x3fc5555555555511ull));
    p = fma_k(r, p, GRM_K(0x3fe000000000000bull));
    p = fma(r, p, 1.0);
    return fma(r, p, 1.0);
}
__device__ __forceinline__ double exp_range(double x, double y) {
    y = x > 1024.0 ? __builtin_huge_val() : y;
    return x < -1075.0 ? 0.0 : y;
}
__device__ __forceinline__ double fexp(double x) {
    const double k = __builtin_rint(x * GRM_K(0x3ff71547652b82feull));
    double r = fma(GRM_K(0xbfe62e42fefa39efull), k, x);
    r = fma(GRM_K(0xbc7abc9e3b39803full), k, r);
    const double p = exp_poly(r);
    return exp_range(x, __builtin_amdgcn_ldexp(p, (int)k));
}
__device__ __forceinline__ double fexp10(double x) {
    const double k = __builtin_rint(x * GRM_K(0x400a934f0979a371ull));
    double r = fma(GRM_K(0xbfd34413509f79ffull), k, x);
    r = fma(GRM_K(0x3c49dc1da994fd21ull), k, r);
    double z = r * GRM_K(0xbcaf48ad494ea3e9ull);
    z = fma(GRM_K(0x40026bb1bbb55516ull), r, z);
    const double p = exp_poly(z);
    return exp_range(x, __builtin_amdgcn_ldexp(p, (int)k));
}

/* ---- natural logarithm ----
 * ocml's log carries a double-double evaluation for < 0.5-ulp results (~90 VALU ops).  flog is the
 * classic fdlibm reduction (x = 2^e m, m in [sqrt(1/2), sqrt(2)), s = (m-1)/(m+1), log m =
 * 2 atanh s as f - f^2/2 + s (f^2/2 + R(s^2)), R a degree-14 minimax polynomial) in ~35 ops, < 1 ulp
 * for positive normal x (tests/test_gpu_probes.py measures it against the host libm); every other x
 * (0, subnormal, negative, inf, NaN) goes to ocml. */
__device__ __forceinline__ double flog(double x) {
    if (!(x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308)) return log(x);
    double m = __builtin_amdgcn_frexp_mant(x); /* [0.5, 1) */
    int e = __builtin_amdgcn_frexp_exp(x);
    if (m < 0.70710678118654752440) {
        m *= 2.0;
        --e;
    }
    const double f = m - 1.0;
    const double s = fdiv(f, 2.0 + f);
    const double z = s * s, w = z * z;
    const double t1 =
        w * fma_k(w, fma_k(w, 1.531383769920937332e-01, 2.222219843214978396e-01), 3.999999999940941908e-01);
    const double t2 = z * fma_k(w,
                                fma_k(w, fma_k(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                                      2.857142874366239149e-01),
                                6.666666666666735130e-01);
    const double r = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)e;
    return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + r) + dk * 1.90821492927058770002e-10)) - f);
}

/* sin(pi x), cos(pi x) for |x| < 2^30 (every argument here is O(1)): exact reduction r = x - n/2,
 * n = rint(2x) (|r| <= 1/4, the fma is exact), Taylor polynomials of sin(pi r)/r and cos(pi r) to
 * degree 16 (truncation < 1e-18 on |r| <= 1/4), quadrant by the low bits of n.  ~32 ops against
 * ocml's ~65 general-argument sincospi; <= 2 ulp (tests/test_gpu_probes.py, against mpmath). */
__device__ __forceinline__ void fsincospi(double x, double &s, double &c) {
    const double n = __builtin_rint(2.0 * x);
    const double r = fma(n, -0.5, x);
    const double t = r * r;
    double ps = 7.952054001475513e-07;
    ps = fma_k(ps, t, -2.1915353447830217e-05);
    ps = fma_k(ps, t, 0.00046630280576761255);
    ps = fma_k(ps, t, -0.0073704309457143504);
    ps = fma_k(ps, t, 0.08214588661112823);
    ps = fma_k(ps, t, -0.5992645293207921);
    ps = fma_k(ps, t, 2.5501640398773455);
    ps = fma_k(ps, t, -5.16771278004997);
    const double sr = fma(r * t, ps, r * 3.141592653589793); /* r (pi + t P(t)) */
    double pc = 4.303069587032947e-06;
    pc = fma_k(pc, t, -0.0001046381049248457);
    pc = fma_k(pc, t, 0.0019295743094039231);
    pc = fma_k(pc, t, -0.02580689139001406);
    pc = fma_k(pc, t, 0.2353306303588932);
    pc = fma_k(pc, t, -1.3352627688545895);
    pc = fma_k(pc, t, 4.0587121264167685);
    pc = fma_k(pc, t, -4.934802200544679);
    const double cr = fma(t, pc, 1.0);
    const int q = (int)n;
    const bool odd = (q & 1) != 0;
    const double a = odd ? cr : sr, b = odd ? sr : cr;
    /* sign flips as xor of the sign bit: s negated for q = 2, 3; c for q = 1, 2 (mod 4) */
    const long long fs = (long long)(q & 2) << 62, fc = (long long)((q + 1) & 2) << 62;
    s = __longlong_as_double(__double_as_longlong(a) ^ fs);
    c = __longlong_as_double(__double_as_longlong(b) ^ fc);
}

/* a / b for a kernel-argument divisor b with host reciprocal ib: one multiply (<= 1 ulp from a / b;
 * only grid / table coordinates go through it, whose interpolants are continuous across cells). */
__device__ __forceinline__ double udiv(double a, double, double ib) { return a * ib; }

/* Kernel-argument block: everything uniform across lanes (lands in SGPRs). */
struct Params {
    int n1, n2;
    double xs1, xs2, xe1, xe2, dx1, dx2; /* x_start/x_stop/dx of dims 1,2 */
    double a, h_slope, r0;
    double n_e_unit, theta_e_unit, b_unit;
    double x1_min, x1_max, d_tau_k, bias_norm;
    double hc_l_min_w, hc_l_min_t, hc_d_l_w, hc_d_l_t;
    double jnu_l_min_t, jnu_d_l_t;
    double spec_l_e_0, th_dx2;
    double i_dx1, i_dx2, hc_i_d_l_w, hc_i_d_l_t, jnu_i_d_l_t; /* host reciprocals of the uniform divisors */
    /* uniform factors of the metric / connection, formed on the host with the device expressions'
     * own operations and order (so the same bits): a^2, a^3, a^4, 1 - h, (1 - h) pi, (1 - h) / (2 pi),
     * (-2 pi pi)(1 - h), -2 a -- fp64 arithmetic on uniform values still costs VALU issue slots */
    double a2, a3, a4, hs1, hs1_pi, th_fac, d2k, m2a;
    const double *zones;    /* [n1*n2][8]: rho,u,u1,u2,u3,B1,B2,B3 (64 B per zone) */
    const double *hotcross; /* [221][81] log10 sigma */
    const double *k2;       /* [201] log K2 */
};

/* the metric's uniform factors of Params from P.a and P.h_slope (host) */
inline void params_metric(Params &P) {
    const double a = P.a, h = P.h_slope;
    P.a2 = a * a;
    P.a3 = P.a2 * a;
    P.a4 = P.a3 * a;
    P.hs1 = 1.0 - h;
    P.hs1_pi = P.hs1 * kPi;
    P.th_fac = P.hs1 / (2.0 * kPi);
    P.d2k = -2.0 * kPi * kPi * P.hs1;
    P.m2a = -2.0 * a;
}

/* ------------------------------------------------------------------------- */
/* Philox4x32-10 per-photon streams (counter = (draw index, photon id))       */
/* ------------------------------------------------------------------------- */
struct Rng {
    uint32_t k0, k1;
    uint64_t id;
    uint32_t ctr, ctr_hi; /* counter words 0, 1: draw index, and the emission slot (0 in transport) */
};

__device__ __forceinline__ void philox_block(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                             uint32_t k1, uint32_t &o0, uint32_t &o1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        /* one 32x32->64 multiply (v_mad_u64_u32) per product instead of mul_lo + mul_hi */
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    o0 = c0;
    o1 = c1;
}

/* uniform double in (0, 1] from 53 random bits */
__device__ __forceinline__ double uniform(Rng &g) {
    uint32_t o0, o1;
    philox_block(g.ctr, g.ctr_hi, (uint32_t)g.id, (uint32_t)(g.id >> 32), g.k0, g.k1, o0,
                 o1);
    ++g.ctr;
    const uint64_t m = ((((uint64_t)o1) << 32) | o0) >> 11;
    return (double)(m + 1) * (1.0 / 9007199254740992.0);
}

/* chi^2(dof) for dof 3..6: -2 ln(prod of dof/2 uniforms) (+ one Box-Muller normal^2 if odd) */
__device__ __forceinline__ double chi_sq(Rng &g, int dof) {
    double prod = uniform(g);
    const int m = dof >> 1;
    for (int i = 1; i < m; ++i) prod *= uniform(g);
    double x = -2.0 * flog(prod);
    if (dof & 1) {
        const double ua = uniform(g);
        const double ub = uniform(g);
        double sb, cb;
        fsincospi(2.0 * ub, sb, cb); /* cos(2 pi ub), exact reduction */
        const double z = sqrt(-2.0 * flog(ua)) * cb;
        x += z * z;
    }
    return x;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t child_id(uint64_t parent_id, uint64_t parent_ctr) {
    return splitmix64(parent_id ^ (0x9E3779B97F4A7C15ull * (parent_ctr + 1)));
}

/* ------------------------------------------------------------------------- */
/* metric (harm_model.cpp:473-530, 1632-1637): one set of transcendentals per  */
/* point, shared by g_cov, the row g^{0mu} and the connection.                */
/* ------------------------------------------------------------------------- */
struct Trig {
    double r1;       /* exp(x1) */
    double s2x, c2x; /* sin/cos(2 pi x2) */
    double sth, cth; /* sin/cos(theta_BL) */
};

/* theta = pi x2 + (1 - h)/2 sin(2 pi x2) (harm_model.cpp gcov/connection): both sincos through
 * sincospi of x2-scaled arguments -- an exact, branch-free range reduction instead of the general
 * one (agreement with sin/cos of the pi-multiplied argument to a few ulp) */
__device__ __forceinline__ void trig_at(const Params &P, const double x[4], Trig &T) {
    T.r1 = fexp(x[1]);
    fsincospi(2.0 * x[2], T.s2x, T.c2x);
    fsincospi(x[2] + P.th_fac * T.s2x, T.sth, T.cth); /* th_fac = (1 - h) / (2 pi) */
}

/* non-zero g_mu,nu of MKS Kerr + g^{00}, g^{01} (g^{02} = g^{03} = 0) */
struct Gcov {
    double g00, g01, g03, g11, g13, g22, g33;
    double gn00, gn01;
};

__device__ __forceinline__ void gcov_from_trig(const Params &P, const Trig &T, Gcov &G) {
    const double r = T.r1 + P.r0;
    const double a = P.a;
    const double sin_theta = fabs(T.sth) + EPS;
    const double cos_theta = T.cth;
    const double s2 = sin_theta * sin_theta;
    const double rho2 = r * r + P.a2 * cos_theta * cos_theta;
    const double rfac = r - P.r0;
    const double hfac = kPi + P.hs1_pi * T.c2x; /* pi + (1 - h) pi cos(2 pi x2) */
    const double irho2 = frcp(rho2);
    const double two_r_rho2 = 2.0 * r * irho2;
    G.g00 = (-1.0 + two_r_rho2);
    G.g01 = two_r_rho2 * rfac;
    G.g03 = P.m2a * r * s2 * irho2; /* -2 a r sin^2 / rho^2 */
    G.g11 = (1.0 + two_r_rho2) * rfac * rfac;
    G.g13 = (-a * s2 * (1.0 + two_r_rho2)) * rfac;
    G.g22 = rho2 * hfac * hfac;
    G.g33 = s2 * (rho2 + P.a2 * s2 * (1.0 + two_r_rho2));
    G.gn00 = -1.0 - 2.0 * r * irho2;
    G.gn01 = 2.0 * irho2;
}

__device__ __forceinline__ void lower(const Gcov &G, const double u[4], double uc[4]) {
    uc[0] = G.g00 * u[0] + G.g01 * u[1] + G.g03 * u[3];
    uc[1] = G.g01 * u[0] + G.g11 * u[1] + G.g13 * u[3];
    uc[2] = G.g22 * u[2];
    uc[3] = G.g03 * u[0] + G.g13 * u[1] + G.g33 * u[3];
}

__device__ __forceinline__ void gcov_full(const Gcov &G, double g[4][4]) {
    g[0][0] = G.g00; g[0][1] = G.g01; g[0][2] = 0.0; g[0][3] = G.g03;
    g[1][0] = G.g01; g[1][1] = G.g11; g[1][2] = 0.0; g[1][3] = G.g13;
    g[2][0] = 0.0;   g[2][1] = 0.0;   g[2][2] = G.g22; g[2][3] = 0.0;
    g[3][0] = G.g03; g[3][1] = G.g13; g[3][2] = 0.0; g[3][3] = G.g33;
}

/* ------------------------------------------------------------------------- */
/* connection (harm_model.cpp:1436-1569): 40 symmetric entries, j<=k;          */
/* entries identically zero (1,0,2) (1,2,3) (2,0,2) (2,2,3) are dropped.       */
/* ------------------------------------------------------------------------- */
struct Conn {
    double c[4][10]; /* [i][tri(j,k)], tri: 00 01 02 03 11 12 13 22 23 33 */
};

/* the products the 40 entries share (computed once per point) */
struct ConnPre {
    double r1, r2, r3, r4, a, a2, a3, a4;
    double sth, cth, sth2, r1sth2, sth4, cth2, cth4, s2th, c2th, a2sth2, a2cth2, a4cth4;
    double dthdx2, d2thdx22, rho2, rho22, rho23, irho2, irho22, irho23, idthdx2, irho23_dthdx2;
    double fac1, fac1_rho23, fac3, i_r1rho23, i_sth;
    double r1f, a2s2d, r1s2d, d2r, fac3f, arcd;
};

__device__ __forceinline__ void connection_pre(const Params &P, const Trig &T, ConnPre &Q) {
    const double r1 = T.r1, r2 = r1 * r1, r3 = r2 * r1, r4 = r3 * r1;
    const double dthdx2 = kPi * (1.0 + P.hs1 * T.c2x);
    const double d2thdx22 = P.d2k * T.s2x; /* -2 pi^2 (1 - h) sin(2 pi x2) */
    const double dthdx22 = dthdx2 * dthdx2;
    const double sth = T.sth, cth = T.cth;
    const double sth2 = sth * sth, r1sth2 = r1 * sth2, sth4 = sth2 * sth2;
    const double cth2 = cth * cth, cth4 = cth2 * cth2;
    const double s2th = 2.0 * sth * cth, c2th = 2.0 * cth2 - 1.0;
    const double a = P.a, a2 = P.a2, a3 = P.a3, a4 = P.a4;
    const double a2sth2 = a2 * sth2, a2cth2 = a2 * cth2, a4cth4 = a4 * cth4;
    const double rho2 = r2 + a2cth2, rho22 = rho2 * rho2, rho23 = rho22 * rho2;
    const double irho2 = frcp(rho2), irho22 = irho2 * irho2, irho23 = irho22 * irho2;
    const double idthdx2 = frcp(dthdx2), irho23_dthdx2 = irho23 * idthdx2;
    const double fac1 = r2 - a2cth2, fac1_rho23 = fac1 * irho23;
    const double fac3 = a2 + r1 * (-2.0 + r1);
    const double i_r1rho23 = frcp(r1) * irho23;
    /* the reference's fac2 = a^2 + 2 r^2 + a^2 cos(2 theta) = 2 rho^2: written through rho^2 below */
    const double i_sth = frcp(sth);
    Q.r1 = r1; Q.r2 = r2; Q.r3 = r3; Q.r4 = r4;
    Q.a = a; Q.a2 = a2; Q.a3 = a3; Q.a4 = a4;
    Q.sth = sth; Q.cth = cth; Q.sth2 = sth2; Q.r1sth2 = r1sth2; Q.sth4 = sth4; Q.cth2 = cth2; Q.cth4 = cth4;
    Q.s2th = s2th; Q.c2th = c2th; Q.a2sth2 = a2sth2; Q.a2cth2 = a2cth2; Q.a4cth4 = a4cth4;
    Q.dthdx2 = dthdx2; Q.d2thdx22 = d2thdx22; Q.rho2 = rho2; Q.rho22 = rho22; Q.rho23 = rho23;
    Q.irho2 = irho2; Q.irho22 = irho22; Q.irho23 = irho23; Q.idthdx2 = idthdx2; Q.irho23_dthdx2 = irho23_dthdx2;
    Q.fac1 = fac1; Q.fac1_rho23 = fac1_rho23; Q.fac3 = fac3; Q.i_r1rho23 = i_r1rho23; Q.i_sth = i_sth;
    /* products shared between entries (reassociated: agreement with the reference's expressions to a
     * few ulp, tests/test_gpu_probes.py::test_connection) */
    Q.r1f = r1 * fac1_rho23;                      /* r fac1 / rho^6 */
    Q.a2s2d = a2 * s2th * dthdx2 * irho22;         /* a^2 sin 2th dth/dx2 / rho^4 */
    Q.r1s2d = r1 * s2th * irho23_dthdx2;           /* r sin 2th / (rho^6 dth/dx2) */
    Q.d2r = dthdx22 * irho2;                       /* (dth/dx2)^2 / rho^2 */
    Q.fac3f = fac3 * fac1 * i_r1rho23;
    Q.arcd = a * r1 * cth * dthdx2 * i_sth * irho22;
}

/* row i of the connection, Gamma^i_{jk} for j <= k in tri order (harm_model.cpp:1436-1569) */
__device__ __forceinline__ void connection_row(const ConnPre &Q, int i, double L[10]) {
    const double r1 = Q.r1, r2 = Q.r2, r3 = Q.r3, r4 = Q.r4, a = Q.a, a2 = Q.a2, a3 = Q.a3, a4 = Q.a4;
    const double sth = Q.sth, cth = Q.cth, sth2 = Q.sth2, r1sth2 = Q.r1sth2, sth4 = Q.sth4, cth2 = Q.cth2,
                 cth4 = Q.cth4;
    const double s2th = Q.s2th, c2th = Q.c2th, a2sth2 = Q.a2sth2, a2cth2 = Q.a2cth2, a4cth4 = Q.a4cth4;
    const double dthdx2 = Q.dthdx2, d2thdx22 = Q.d2thdx22, rho2 = Q.rho2, rho22 = Q.rho22, rho23 = Q.rho23;
    const double irho2 = Q.irho2, irho22 = Q.irho22, irho23 = Q.irho23, idthdx2 = Q.idthdx2,
                 irho23_dthdx2 = Q.irho23_dthdx2;
    const double fac1 = Q.fac1, fac1_rho23 = Q.fac1_rho23, fac3 = Q.fac3, i_r1rho23 = Q.i_r1rho23, i_sth = Q.i_sth;
    const double r1f = Q.r1f, a2s2d = Q.a2s2d, r1s2d = Q.r1s2d, d2r = Q.d2r, fac3f = Q.fac3f, arcd = Q.arcd;
    if (i == 0) {
        L[0] = 2.0 * r1f;
        L[1] = (2.0 * r1 + rho2) * r1f;
        L[2] = -r1 * a2s2d;
        L[3] = -2.0 * a * sth2 * r1f;
        L[4] = 2.0 * r2 * (r4 + r1 * fac1 - a4cth4) * irho23;
        L[5] = -r2 * a2s2d;
        L[6] = a * r1 * (-r1 * (r3 + 2.0 * fac1) + a4cth4) * sth2 * irho23;
        L[7] = -2.0 * r2 * d2r;
        L[8] = a * r1sth2 * a2s2d;
        L[9] = 2.0 * r1sth2 * (-r1 * rho22 + a2sth2 * fac1) * irho23;
    } else if (i == 1) {
        L[0] = fac3f;
        L[1] = fac1 * (-2.0 * r1 + a2sth2) * irho23;
        L[2] = 0.0;
        L[3] = -a * sth2 * fac3f;
        L[4] = (r4 * (-2.0 + r1) * (1.0 + r1) +
                a2 * (a2 * r1 * (1.0 + 3.0 * r1) * cth4 + a4cth4 * cth2 + r3 * sth2 +
                      r1 * cth2 * (2.0 * r1 + 3.0 * r3 - a2sth2))) *
               irho23;
        L[5] = -0.5 * rho2 * a2s2d; /* -a^2 dth/dx2 sin 2th / (2 rho^2) */
        L[6] = a * sth2 * (a4 * r1 * cth4 + r2 * (2.0 * r1 + r3 - a2sth2) + a2cth2 * (2.0 * r1 * (-1.0 + r2) + a2sth2)) *
               irho23;
        L[7] = -fac3 * d2r;
        L[8] = 0.0;
        L[9] = -fac3 * sth2 * (r1 * rho22 - a2 * fac1 * sth2) * i_r1rho23;
    } else if (i == 2) {
        L[0] = -a2 * r1s2d;
        L[1] = r1 * L[0];
        L[2] = 0.0;
        L[3] = a * (a2 + r2) * r1s2d;
        L[4] = r2 * L[0];
        L[5] = r2 * irho2;
        L[6] = (a * r1 * cth * sth * (r3 * (2.0 + r1) + a2 * (2.0 * r1 * (1.0 + r1) * cth2 + a2 * cth4 + 2.0 * r1sth2))) *
               irho23_dthdx2;
        L[7] = -a2 * cth * sth * dthdx2 * irho2 + d2thdx22 * idthdx2;
        L[8] = 0.0;
        L[9] = -cth * sth * (rho23 + a2sth2 * rho2 * (r1 * (4.0 + r1) + a2cth2) + 2.0 * r1 * a4 * sth4) * irho23_dthdx2;
    } else {
        L[0] = a * fac1_rho23;
        L[1] = a * r1f;
        L[2] = -2.0 * arcd;
        L[3] = -a2sth2 * fac1_rho23;
        L[4] = a * r1 * r1f;
        /* ifac2^2 = irho2^2 / 4 */
        L[5] = -0.5 * (a2 + 2.0 * r1 * (2.0 + r1) + a2 * c2th) * arcd;
        L[6] = r1 * (r1 * rho22 - a2sth2 * fac1) * irho23;
        L[7] = -a * r1 * d2r;
        L[8] = dthdx2 * (rho22 * cth * i_sth + a2 * r1 * s2th) * irho22; /* fac2^2 / 4 = rho^4 */
        L[9] = (-a * r1sth2 * rho22 + a3 * sth4 * fac1) * irho23;
    }
}

__device__ __forceinline__ void connection(const Params &P, const Trig &T, Conn &C) {
    ConnPre Q;
    connection_pre(P, T, Q);
#pragma unroll
    for (int i = 0; i < 4; ++i) connection_row(Q, i, C.c[i]);
}

/* dk^i/dlambda = -Gamma^i_{jk} k^j k^k (harm_model.cpp:1255-1262, 1578-1586) */
__device__ __forceinline__ double geo_rhs(const Conn &C, int i, const double k[4]) {
    const double *L = C.c[i];
    double d = -2.0 * (k[0] * (L[1] * k[1] + L[2] * k[2] + L[3] * k[3]) + k[1] * (L[5] * k[2] + L[6] * k[3]) +
                       L[8] * k[2] * k[3]);
    d -= (L[0] * k[0] * k[0] + L[4] * k[1] * k[1] + L[7] * k[2] * k[2] + L[9] * k[3] * k[3]);
    return d;
}

__device__ __forceinline__ void init_dkdlam(const Params &P, const double x[4], const double k[4], double dk[4]) {
    Trig T;
    trig_at(P, x, T);
    Conn C;
    connection(P, T, C);
#pragma unroll
    for (int i = 0; i < 4; ++i) dk[i] = geo_rhs(C, i, k);
}

/* harm_model.cpp:1620-1630 */
__device__ __forceinline__ double step_size(const Params &P, const double x[4], const double k[4]) {
    /* 1 / (|a / b| + EPS) = b / d with b = |k| + EPS > 0 and d = |a| + EPS b > 0, so
     * dl = 1 / (b1/d1 + b2/d2 + b3/d3) = d1 d2 d3 / (b1 d2 d3 + b2 d1 d3 + b3 d1 d2): one division
     * instead of the reference's seven (same value to a few ulp; d >= 1e-40 b >= 1e-80 and every
     * product stays far inside the fp64 range) -- it sits on the serial chain of every step */
    const double b1 = fabs(k[1]) + EPS, b2 = fabs(k[2]) + EPS, b3 = fabs(k[3]) + EPS;
    const double d1 = fabs(STEP_EPS * x[1]) + EPS * b1;
    const double d2 = fabs(STEP_EPS * fmin(x[2], P.xe2 - x[2])) + EPS * b2;
    const double d3 = STEP_EPS + EPS * b3;
    const double d23 = d2 * d3, d12 = d1 * d2;
    return fdiv(d1 * d23, fma(b1, d23, fma(b2, d1 * d3, b3 * d12)));
}

/* One attempted push of length dl (body of harm_model.cpp:1230-1277).  Returns the fail
 * predicate of :1279 and the new energy e_1; leaves Trig and Gcov at the new x in T, G. */
/* push_attempt's halves: the half-step kick (x, k advanced, kp the predictor) ... */
__device__ __forceinline__ void push_kick(double x[4], double k[4], const double dk[4], double dl, double kp[4]) {
    const double dl_2 = 0.5 * dl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double d = dk[i] * dl_2;
        k[i] += d;
        kp[i] = k[i] + d;
        x[i] += k[i] * dl;
    }
}

/* ... and, with the connection at the new x, the corrector iterations and the energy check
 * (g00, g01, g03 of the metric there) */
__device__ __forceinline__ bool push_finish(const Conn &C, double k[4], double kp[4], double dk[4], double dl,
                                            double e_0_s, double g00, double g01, double g03, double &e_1) {
    const double dl_2 = 0.5 * dl;
    double err;
    int iter = 0;
    do {
        ++iter;
        const double kc[4] = {kp[0], kp[1], kp[2], kp[3]};
        err = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            dk[i] = geo_rhs(C, i, kc);
            kp[i] = k[i] + dl_2 * dk[i];
            err += fratio_tol(kc[i] - kp[i], kp[i] + EPS);
        }
    } while (err > E_TOL && iter < MAX_ITER);
#pragma unroll
    for (int i = 0; i < 4; ++i) k[i] = kp[i];
    e_1 = -(k[0] * g00 + k[1] * g01 + k[3] * g03);
    /* |(e_1 - e_0_s) / e_0_s| > 1e-4 without the divide: same outcome for e_0_s = 0 (0/0 = NaN
     * fails neither test, x/0 = inf passes both) and NaN operands */
    const bool err_e = fabs(e_1 - e_0_s) > 1.0e-4 * fabs(e_0_s);
    return (err_e || err > E_TOL || isnan(err) || isinf(err));
}

/* One attempted push of length dl (body of harm_model.cpp:1230-1277).  Returns the fail
 * predicate of :1279 and the new energy e_1; leaves Trig and Gcov at the new x in T, G. */
__device__ __forceinline__ bool push_attempt(const Params &P, double x[4], double k[4], double dk[4], double e_0_s,
                                             double dl, double &e_1, Trig &T, Gcov &G) {
    double kp[4];
    push_kick(x, k, dk, dl, kp);
    trig_at(P, x, T);
    Conn C;
    connection(P, T, C);
    gcov_from_trig(P, T, G);
    return push_finish(C, k, kp, dk, dl, e_0_s, G.g00, G.g01, G.g03, e_1);
}

/* ---- quad-parallel push (one photon per quad of lanes: the serial chain of a lone photon) ----
 * A single wave issues a wave-instruction every ~4.4 cycles whether 1 or 64 lanes are active, so a
 * push that every lane makes identically pays the full instruction count.  Here the four lanes of a
 * quad hold the same attempt and lane q = lane & 3 owns row q of the connection: the rows are formed
 * in four exec-masked blocks (the same instructions as one lane forming all four), and the corrector
 * -- two passes of four row contractions and four tolerance ratios, ~40 % of an attempt -- runs ONE
 * row per lane on a uniform instruction stream; k and the ratios are exchanged inside the quad by
 * DPP quad_perm moves (no LDS, no SGPR round trip).  Each row is contracted with the reference's own
 * expression and the ratios are summed in its order (e_0 + e_1) + e_2 + e_3, so every lane ends with
 * the bits of push_attempt. */
template <int I>
__device__ __forceinline__ double quad_bcast(double v) {
    constexpr int ctl = I | (I << 2) | (I << 4) | (I << 6); /* quad_perm [I, I, I, I] */
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, ctl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), ctl, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

/* v[q] for the lane's quad position q (three selects per 32-bit half) */
__device__ __forceinline__ double quad_pick(const double v[4], int q) {
    const double lo = (q & 1) ? v[1] : v[0], hi = (q & 1) ? v[3] : v[2];
    return (q & 2) ? hi : lo;
}

/* geo_rhs of one row (the same expression, harm_model.cpp:1255-1262) */
__device__ __forceinline__ double geo_rhs_row(const double L[10], const double k[4]) {
    double d = -2.0 * (k[0] * (L[1] * k[1] + L[2] * k[2] + L[3] * k[3]) + k[1] * (L[5] * k[2] + L[6] * k[3]) +
                       L[8] * k[2] * k[3]);
    d -= (L[0] * k[0] * k[0] + L[4] * k[1] * k[1] + L[7] * k[2] * k[2] + L[9] * k[3] * k[3]);
    return d;
}

/* row q from two exec-masked blocks of two rows each (lanes 0-1 form rows 0, 1; lanes 2-3 rows 2, 3):
 * the rows of a block interleave, and one select per 32-bit half picks the lane's row (20 selects) */
__device__ __forceinline__ void connection_quad_half(const Params &P, const Trig &T, int q, double L[10]) {
    ConnPre Q;
    connection_pre(P, T, Q);
    double A[10], B[10];
    if (q < 2) {
        connection_row(Q, 0, A);
        connection_row(Q, 1, B);
    } else {
        connection_row(Q, 2, A);
        connection_row(Q, 3, B);
    }
#pragma unroll
    for (int j = 0; j < 10; ++j) L[j] = (q & 1) ? B[j] : A[j];
}

/* push_attempt on a quad (q = lane & 3; x, k, dk, e_0_s identical over the quad on entry and exit);
 * row q of the connection reaches lane q from two exec-masked blocks of two rows each (four divergent
 * one-row blocks and a 60-select pick from all four rows were measured slower: DESIGN.md §4.2) */
__device__ __forceinline__ bool push_attempt_quad(const Params &P, double x[4], double k[4], double dk[4],
                                                  double e_0_s, double dl, double &e_1, Trig &T, Gcov &G, int q) {
    double kp[4];
    push_kick(x, k, dk, dl, kp);
    trig_at(P, x, T);
    double L[10];
    connection_quad_half(P, T, q, L);
    gcov_from_trig(P, T, G);
    const double dl_2 = 0.5 * dl;
    const double kq = quad_pick(k, q); /* the half-kicked k^q */
    double kcq = quad_pick(kp, q);     /* k_cont^q */
    double kc[4] = {kp[0], kp[1], kp[2], kp[3]};
    double err, dkq;
    int iter = 0;
    do {
        ++iter;
        dkq = geo_rhs_row(L, kc);
        const double kpq = kq + dl_2 * dkq;
        const double eq = fratio_tol(kcq - kpq, kpq + EPS);
        err = ((0.0 + quad_bcast<0>(eq)) + quad_bcast<1>(eq)) + quad_bcast<2>(eq);
        err += quad_bcast<3>(eq);
        kc[0] = quad_bcast<0>(kpq);
        kc[1] = quad_bcast<1>(kpq);
        kc[2] = quad_bcast<2>(kpq);
        kc[3] = quad_bcast<3>(kpq);
        kcq = kpq;
    } while (err > E_TOL && iter < MAX_ITER);
#pragma unroll
    for (int i = 0; i < 4; ++i) k[i] = kc[i];
    dk[0] = quad_bcast<0>(dkq);
    dk[1] = quad_bcast<1>(dkq);
    dk[2] = quad_bcast<2>(dkq);
    dk[3] = quad_bcast<3>(dkq);
    e_1 = -(k[0] * G.g00 + k[1] * G.g01 + k[3] * G.g03);
    const bool err_e = fabs(e_1 - e_0_s) > 1.0e-4 * fabs(e_0_s);
    return (err_e || err > E_TOL || isnan(err) || isinf(err));
}

/* Per-lane spill slot for the push backup, laid out [component][lane] so that a wave's
 * accesses are consecutive 8-B words (conflict-free ds_read_b64 / ds_write_b64).  The
 * transport kernel points it at LDS; the probe kernel at a private array. */
struct Slot {
    double *p;
    int stride;
    __device__ __forceinline__ double &operator[](int i) const { return p[i * stride]; }
};

/* push_photon (harm_model.cpp:1217-1289) without recursion: a depth-first walk of the
 * halving tree.  Bit k of `pend` marks a pending second half at depth k.  Sub-step length
 * dl * 2^-depth is exact (power-of-two scaling), as the reference's 0.5*dl chain is.
 * bk: 12-double backup of (x, k, dk) at the start of the current attempt. */
__device__ __forceinline__ void push_photon(const Params &P, double x[4], double k[4], double dk[4], double &e_0_s,
                                            double dl, const Slot &bk) {
    int depth = 0;
    uint32_t pend = 0;
    while (true) {
        if (!(x[1] < P.xs1)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                bk[i] = x[i];
                bk[4 + i] = k[i];
                bk[8 + i] = dk[i];
            }
            double e_1;
            Trig T;
            Gcov G;
            const bool fail = push_attempt(P, x, k, dk, e_0_s, ldexp(dl, -depth), e_1, T, G);
            if (fail && depth < MAX_SUBDIV) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    x[i] = bk[i];
                    k[i] = bk[4 + i];
                    dk[i] = bk[8 + i];
                }
                ++depth;
                pend |= 1u << depth;
                continue;
            }
            e_0_s = e_1;
        }
        if (pend == 0) break;
        depth = 31 - __builtin_clz(pend);
        pend &= ~(1u << depth);
    }
}

/* ------------------------------------------------------------------------- */
/* fluid (harm_model.cpp:595-671, x_to_ij 1406-1434, interp_scalar 1646-1656) */
/* ------------------------------------------------------------------------- */
struct Fluid {
    double n_e, theta_e, b;
    double u_con[4], u_cov[4], b_con[4], b_cov[4];
};

/* cell-centred zone index and bilinear weights of x (x_to_ij, harm_model.cpp:1406-1434, with the
 * edge clamp of interp_scalar); false = out of the grid */
__device__ __forceinline__ bool zone_index(const Params &P, const double x[4], int &i, int &j, double &di, double &dj) {
    if (x[1] < P.xs1 || x[1] > P.xe1 || x[2] < P.xs2 || x[2] > P.xe2) {
        i = j = 0; /* a valid zone, so callers may load unconditionally and select afterwards */
        di = dj = 0.0;
        return false;
    }
    const double t1 = udiv(x[1] - P.xs1, P.dx1, P.i_dx1), t2 = udiv(x[2] - P.xs2, P.dx2, P.i_dx2);
    i = (int)(t1 - 0.5 + 1000) - 1000;
    j = (int)(t2 - 0.5 + 1000) - 1000;
    if (i < 0) {
        i = 0;
        di = 0.0;
    } else if (i > P.n1 - 2) {
        i = P.n1 - 2;
        di = 1.0;
    } else {
        di = t1 - (i + 0.5);
    }
    if (j < 0) {
        j = 0;
        dj = 0.0;
    } else if (j > P.n2 - 2) {
        j = P.n2 - 2;
        dj = 1.0;
    } else {
        dj = t2 - (j + 0.5);
    }
    return true;
}

/* the 4 zones around x: (i,j),(i,j+1) and (i+1,j),(i+1,j+1) are two contiguous 128-B runs of the
 * zone-major [n1][n2][8] field array, 8 x 16-B loads each */
struct ZoneFetch {
    double2 v[16];
};

__device__ __forceinline__ void zone_fetch(const Params &P, const double x[4], ZoneFetch &Z) {
    int i, j;
    double di, dj;
    zone_index(P, x, i, j, di, dj); /* out of the grid: zone (0, 0), result unused */
    const double2 *z0 = reinterpret_cast<const double2 *>(P.zones + ((size_t)i * P.n2 + j) * 8);
    const double2 *z1 = reinterpret_cast<const double2 *>(P.zones + ((size_t)(i + 1) * P.n2 + j) * 8);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        Z.v[q] = z0[q];
        Z.v[8 + q] = z1[q];
    }
}

/* get_fluid_params (harm_model.cpp:595-671) from fetched zones */
__device__ __forceinline__ void fluid_from(const Params &P, const double x[4], const Gcov &G, const ZoneFetch &Z,
                                           Fluid &F) {
    int i, j;
    double di, dj;
    const bool in_grid = zone_index(P, x, i, j, di, dj);
    const double c0 = (1.0 - di) * (1.0 - dj), c1 = (1.0 - di) * dj, c2 = di * (1.0 - dj), c3 = di * dj;
    double v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const double2 a = Z.v[q], b = Z.v[q + 4], c = Z.v[8 + q], d = Z.v[12 + q];
        v[2 * q] = a.x * c0 + b.x * c1 + c.x * c2 + d.x * c3;
        v[2 * q + 1] = a.y * c0 + b.y * c1 + c.y * c2 + d.y * c3;
    }
    const double rho = v[0], uu = v[1];
    F.n_e = rho * P.n_e_unit;
    F.theta_e = fdiv(uu, rho) * P.theta_e_unit;
    const double vc1 = v[2], vc2 = v[3], vc3 = v[4];
    const double bp1 = v[5], bp2 = v[6], bp3 = v[7];
    const double vdv = G.g11 * vc1 * vc1 + G.g13 * vc1 * vc3 + G.g22 * vc2 * vc2 + G.g13 * vc3 * vc1 + G.g33 * vc3 * vc3;
    const double vfac = sqrt(-frcp(G.gn00) * (1.0 + fabs(vdv)));
    F.u_con[0] = -vfac * G.gn00;
    F.u_con[1] = vc1 - vfac * G.gn01;
    F.u_con[2] = vc2;
    F.u_con[3] = vc3;
    lower(G, F.u_con, F.u_cov);
    const double udb = F.u_cov[1] * bp1 + F.u_cov[2] * bp2 + F.u_cov[3] * bp3;
    const double iu0 = frcp(F.u_con[0]);
    F.b_con[0] = udb;
    F.b_con[1] = (bp1 + F.u_con[1] * udb) * iu0;
    F.b_con[2] = (bp2 + F.u_con[2] * udb) * iu0;
    F.b_con[3] = (bp3 + F.u_con[3] * udb) * iu0;
    lower(G, F.b_con, F.b_cov);
    F.b = sqrt(F.b_con[0] * F.b_cov[0] + F.b_con[1] * F.b_cov[1] + F.b_con[2] * F.b_cov[2] + F.b_con[3] * F.b_cov[3]) *
          P.b_unit;
    if (!in_grid) {
        /* out of grid: n_e = 0; the reference leaves the rest unset, we zero it (so does the oracle).
         * Computed on zone (0, 0) and discarded, branch-free (no per-lane stack copies) */
        F.n_e = F.theta_e = F.b = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) F.u_con[q] = F.u_cov[q] = F.b_con[q] = F.b_cov[q] = 0.0;
    }
}

__device__ __forceinline__ void fluid_params(const Params &P, const double x[4], const Gcov &G, Fluid &F) {
    ZoneFetch Z;
    zone_fetch(P, x, Z);
    fluid_from(P, x, G, Z, F);
}

/* ------------------------------------------------------------------------- */
/* radiation (radiation.cpp:59-146), hotcross lookup (hotcross.cpp:81-106),   */
/* synchrotron (jnu_mixed.cpp:75-111, 150-158)                                */
/* ------------------------------------------------------------------------- */
__device__ __forceinline__ double bk_angle(const double k[4], const Fluid &F, double b_unit) {
    if (F.b == 0.0) return kPi / 2.0;
    const double k_ = fabs(k[0] * F.u_cov[0] + k[1] * F.u_cov[1] + k[2] * F.u_cov[2] + k[3] * F.u_cov[3]);
    double mu = (k[0] * F.b_cov[0] + k[1] * F.b_cov[1] + k[2] * F.b_cov[2] + k[3] * F.b_cov[3]) / (k_ * F.b / b_unit);
    mu = fmin(fmax(mu, -1.0), 1.0);
    return acos(mu);
}

/* sin(bk_angle): the synchrotron emissivity only needs sin(theta) = sqrt(1 - mu^2), theta in
 * [0, pi]; saves the acos + sin pair (theta = pi/2 when b = 0, as bk_angle) */
__device__ __forceinline__ double bk_sin(const double k[4], const Fluid &F, double b_unit) {
    if (F.b == 0.0) return 1.0;
    const double k_ = fabs(k[0] * F.u_cov[0] + k[1] * F.u_cov[1] + k[2] * F.u_cov[2] + k[3] * F.u_cov[3]);
    double mu = fdiv((k[0] * F.b_cov[0] + k[1] * F.b_cov[1] + k[2] * F.b_cov[2] + k[3] * F.b_cov[3]) * b_unit, k_ * F.b);
    mu = fmin(fmax(mu, -1.0), 1.0);
    return sqrt((1.0 - mu) * (1.0 + mu));
}

__device__ __forceinline__ double fluid_nu(const double k[4], const Fluid &F) {
    const double energy = -(k[0] * F.u_cov[0] + k[1] * F.u_cov[1] + k[2] * F.u_cov[2] + k[3] * F.u_cov[3]);
    return energy * (ME * CL * CL / HPL);
}

__device__ __forceinline__ double hc_klein_nishina(double w) { /* hotcross.cpp:144-151 */
    if (w < 1.0e-3) return (1.0 - 2.0 * w);
    return (3.0 / 4.0) * (2.0 / (w * w) + (1.0 / (2.0 * w) - (1.0 + w) / (w * w * w)) * log(1.0 + 2.0 * w) +
                          (1.0 + w) / ((1.0 + 2.0 * w) * (1.0 + 2.0 * w)));
}

/* e^x K_2(x) = int_0^inf exp(-x (cosh t - 1)) cosh 2t dt, trapezoid rule (spectrally accurate
 * for this analytic integrand); double-precision replacement for std::cyl_bessel_k (Q5). */
__device__ __noinline__ double k2_scaled(double x) {
    const double h = 1.0 / 32.0;
    double sum = 0.5;
    for (int n = 1; n < 20000; ++n) {
        const double t = n * h;
        const double term = exp(-x * (cosh(t) - 1.0)) * cosh(2.0 * t);
        sum += term;
        if (term < 1.0e-18 * sum) break;
    }
    return sum * h;
}

/* total_compton_cross_num (hotcross.cpp:108-142): rare fallback outside the table */
__device__ __noinline__ double hotcross_num(double w, double theta_e) {
    if (isnan(w)) return 0.0;
    if (theta_e < HC_MIN_T && w < HC_MIN_W) return SIGMA_THOMSON;
    if (theta_e < HC_MIN_T) return hc_klein_nishina(w) * SIGMA_THOMSON;
    const double k2f = (theta_e > 1.0e-2) ? k2_scaled(1.0 / theta_e) : sqrt(kPi * theta_e / 2.0);
    double cross = 0.0;
    for (double mu_e = -1.0 + 0.5 * HC_D_MU_E; mu_e < 1.0; mu_e += HC_D_MU_E) {
        for (double g = 1.0 + 0.5 * theta_e * HC_D_GAMMA_E; g < 1.0 + HC_MAX_GAMMA * theta_e;
             g += theta_e * HC_D_GAMMA_E) {
            const double f = 0.5 * ((g * sqrt(g * g - 1.) / (theta_e * k2f)) * exp(-(g - 1.) / theta_e));
            const double v = sqrt(g * g - 1.0) / g;
            const double bc = hc_klein_nishina(w * g * (1.0 - mu_e * v)) * (1.0 - mu_e * v);
            cross += theta_e * HC_D_MU_E * HC_D_GAMMA_E * bc * f;
        }
    }
    return cross * SIGMA_THOMSON;
}

/* ln_te = ln(theta_e), shared with k2_eval */
__device__ __forceinline__ double hotcross_lkup(const Params &P, double w, double theta_e, double ln_te) {
    if (w * theta_e < 1.0e-6) return SIGMA_THOMSON;
    if (theta_e < HC_MIN_T) return hc_klein_nishina(w) * SIGMA_THOMSON;
    if (w <= HC_MIN_W || w >= HC_MAX_W || theta_e <= HC_MIN_T || theta_e >= HC_MAX_T) return hotcross_num(w, theta_e);
    const double fi = (log10(w) - P.hc_l_min_w) / P.hc_d_l_w;
    const double fj = (ln_te * kLog10E - P.hc_l_min_t) / P.hc_d_l_t;
    const int i = (int)fi, j = (int)fj;
    const double d_i = fi - i, d_j = fj - j;
    const double *t = P.hotcross + (size_t)i * (HC_N_T + 1) + j;
    const double t00 = t[0], t01 = t[1], t10 = t[HC_N_T + 1], t11 = t[HC_N_T + 2];
    const double lc =
        (1.0 - d_i) * (1.0 - d_j) * t00 + d_i * (1.0 - d_j) * t10 + (1.0 - d_i) * d_j * t01 + d_i * d_j * t11;
    return exp10(lc);
}

__device__ __forceinline__ double hotcross_lkup(const Params &P, double w, double theta_e) {
    return hotcross_lkup(P, w, theta_e, log(theta_e));
}

__device__ __forceinline__ double k2_eval(const Params &P, double theta_e, double ln_te) {
    if (theta_e < THETA_E_MIN) return 0.0;
    if (theta_e > JNU_MAX_T) return 2.0 * theta_e * theta_e;
    double d_i = (ln_te - P.jnu_l_min_t) / P.jnu_d_l_t;
    const int i = min((int)d_i, GRM_N_E_SAMP - 1); /* theta_e == 100 exactly: stay in the table */
    d_i -= i;
    return exp((1.0 - d_i) * P.k2[i] + d_i * P.k2[i + 1]);
}

__device__ __forceinline__ double k2_eval(const Params &P, double theta_e) { return k2_eval(P, theta_e, log(theta_e)); }

/* jnu_mixed::synch with sin(theta) and ln(theta_e) supplied */
__device__ __forceinline__ double synch_s(const Params &P, double nu, double n_e, double theta_e, double b,
                                          double sin_theta, double ln_te) {
    if (theta_e < THETA_E_MIN) return 0.0;
    const double k2 = k2_eval(P, theta_e, ln_te);
    const double nu_c = EE * b / (2.0 * kPi * ME * CL);
    const double nu_s = (2.0 / 9.0) * nu_c * theta_e * theta_e * sin_theta;
    if (nu > 1.0e12 * nu_s) return 0.0;
    const double x = nu / nu_s;
    const double xp = cbrt(x);
    const double xx = sqrt(x) + JNU_CST * sqrt(xp);
    const double f = xx * xx;
    return (kSqrt2 * kPi * EE * EE * n_e * nu_s / (3.0 * CL * k2)) * f * exp(-xp);
}

__device__ __forceinline__ double synch(const Params &P, double nu, double n_e, double theta_e, double b,
                                        double theta) {
    return synch_s(P, nu, n_e, theta_e, b, sin(theta), log(theta_e));
}

__device__ __forceinline__ double alpha_inv_scatt(const Params &P, double nu, double theta_e, double n_e,
                                                  double ln_te) {
    const double e_g = HPL * nu / (ME * CL * CL);
    const double kappa = hotcross_lkup(P, e_g, theta_e, ln_te) / MP;
    return nu * kappa * n_e * MP;
}

__device__ __forceinline__ double alpha_inv_scatt(const Params &P, double nu, double theta_e, double n_e) {
    return alpha_inv_scatt(P, nu, theta_e, n_e, log(theta_e));
}

/* alpha_inv_abs with sin(theta) and ln(theta_e) supplied */
__device__ __forceinline__ double alpha_inv_abs_s(const Params &P, double nu, double theta_e, double n_e, double b,
                                                  double sin_theta, double ln_te) {
    const double j = synch_s(P, nu, n_e, theta_e, b, sin_theta, ln_te) / (nu * nu);
    const double x = HPL * nu / (ME * CL * CL * theta_e);
    double b_nu;
    if (x < 1.0e-3)
        b_nu = (2.0 * HPL / (CL * CL)) / (x / 24.0 * (24.0 + x * (12.0 + x * (4.0 + x))));
    else
        b_nu = (2.0 * HPL / (CL * CL)) / (exp(x) - 1.0);
    return j / (b_nu + 1.0e-100);
}

__device__ __forceinline__ double alpha_inv_abs(const Params &P, double nu, double theta_e, double n_e, double b,
                                                double theta) {
    return alpha_inv_abs_s(P, nu, theta_e, n_e, b, sin(theta), log(theta_e));
}

/* alpha_inv_scatt + alpha_inv_abs together (radiation.cpp:103-146, hotcross.cpp:81-106,
 * jnu_mixed.cpp:75-111), the formulas of the separate functions above (constant factors folded,
 * divisions through fdiv: agreement to a few ulp, tests/test_gpu_probes.py), scheduled for one wave per
 * SIMD: both table indices are formed first and all six table loads (hotcross 4, K2 2) are issued
 * unconditionally (index 0 when a branch does not use the table), so their L2 latency overlaps
 * sin(theta), the synchrotron and Planck terms instead of being exposed twice in a row. */
__device__ __forceinline__ void radiation_coeffs(const Params &P, const double k[4], const Fluid &F, double nu,
                                                 double &a_s, double &a_a) {
    const double theta_e = F.theta_e, n_e = F.n_e, b = F.b;
    const double ln_te = flog(theta_e);
    /* hotcross lookup index (hotcross.cpp:82-100) */
    const double w = nu * (HPL / (ME * CL * CL));
    const bool hc_thomson = w * theta_e < 1.0e-6;
    const bool hc_kn = !hc_thomson && theta_e < HC_MIN_T;
    const bool hc_num =
        !hc_thomson && !hc_kn && (w <= HC_MIN_W || w >= HC_MAX_W || theta_e <= HC_MIN_T || theta_e >= HC_MAX_T);
    const bool hc_table = !hc_thomson && !hc_kn && !hc_num;
    double fi = 0.0, fj = 0.0;
    if (hc_table) {
        fi = udiv(flog(w) * kLog10E - P.hc_l_min_w, P.hc_d_l_w, P.hc_i_d_l_w);
        fj = udiv(ln_te * kLog10E - P.hc_l_min_t, P.hc_d_l_t, P.hc_i_d_l_t);
    }
    const int i = hc_table ? (int)fi : 0, j = hc_table ? (int)fj : 0;
    /* K2 index (jnu_mixed.cpp:102-111, 150-158) */
    const bool k2_table = !(theta_e < THETA_E_MIN) && !(theta_e > JNU_MAX_T);
    double dk = k2_table ? udiv(ln_te - P.jnu_l_min_t, P.jnu_d_l_t, P.jnu_i_d_l_t) : 0.0;
    const int ik = k2_table ? min((int)dk, GRM_N_E_SAMP - 1) : 0;
    const double *t = P.hotcross + (size_t)i * (HC_N_T + 1) + j;
    const double t00 = t[0], t01 = t[1], t10 = t[HC_N_T + 1], t11 = t[HC_N_T + 2];
    const double k2a = P.k2[ik], k2b = P.k2[ik + 1];
    /* table-independent work while the loads are in flight: sin(theta) (bk_sin), the synchrotron
     * frequency terms, the Planck denominator */
    const double sin_theta = bk_sin(k, F, P.b_unit);
    const double nu_c = b * (EE / (2.0 * kPi * ME * CL));
    const double nu_s = (2.0 / 9.0) * nu_c * theta_e * theta_e * sin_theta;
    const double x = fdiv(nu, nu_s);
    const double xp = cbrt(x);
    const double sxp = sqrt(xp);
    const double xx = xp * sxp + JNU_CST * sxp; /* sqrt(x) = xp^(3/2) */
    const double f = xx * xx;
    const double xb = fdiv(w, theta_e);
    double b_nu;
    if (xb < 1.0e-3)
        b_nu = fdiv(2.0 * HPL / (CL * CL), xb * (1.0 / 24.0) * (24.0 + xb * (12.0 + xb * (4.0 + xb))));
    else
        b_nu = fdiv(2.0 * HPL / (CL * CL), fexp(xb) - 1.0);
    /* scattering: kappa_es * nu * n_e * m_p */
    double sigma;
    if (hc_thomson) {
        sigma = SIGMA_THOMSON;
    } else if (hc_kn) {
        sigma = hc_klein_nishina(w) * SIGMA_THOMSON;
    } else if (hc_num) {
        sigma = hotcross_num(w, theta_e);
    } else {
        const double d_i = fi - i, d_j = fj - j;
        const double lc =
            (1.0 - d_i) * (1.0 - d_j) * t00 + d_i * (1.0 - d_j) * t10 + (1.0 - d_i) * d_j * t01 + d_i * d_j * t11;
        sigma = fexp10(lc);
    }
    a_s = nu * sigma * n_e; /* nu kappa n_e m_p, kappa = sigma / m_p */
    /* absorption: j_nu / nu^2 / (B_nu / nu^3) */
    double jnu = 0.0;
    if (!(theta_e < THETA_E_MIN) && !(nu > 1.0e12 * nu_s)) {
        /* exp(-x^(1/3)) / K2 as one exponential: K2 = exp(table lerp), or 2 theta_e^2 above the
         * table (then through log -- rare) */
        double l_k2;
        if (theta_e > JNU_MAX_T) {
            l_k2 = log(2.0 * theta_e * theta_e);
        } else {
            dk -= ik;
            l_k2 = (1.0 - dk) * k2a + dk * k2b;
        }
        jnu = ((kSqrt2 * kPi * EE * EE / (3.0 * CL)) * n_e * nu_s) * f * fexp(-xp - l_k2);
    }
    a_a = fdiv(jnu, nu * nu * (b_nu + 1.0e-100));
}

/* ------------------------------------------------------------------------- */
/* scattering: tetrads.cpp:46-194, proba.cpp:30-215, harm_model.cpp:1071-1215 */
/* ------------------------------------------------------------------------- */
/* g(a, b) with the sparse MKS metric (zero entries skipped) */
__device__ __forceinline__ double gdot(const Gcov &G, const double a[4], const double b[4]) {
    return a[0] * (G.g00 * b[0] + G.g01 * b[1] + G.g03 * b[3]) + a[1] * (G.g01 * b[0] + G.g11 * b[1] + G.g13 * b[3]) +
           a[2] * (G.g22 * b[2]) + a[3] * (G.g03 * b[0] + G.g13 * b[1] + G.g33 * b[3]);
}

__device__ __forceinline__ void t_normalize(double v[4], const Gcov &G) {
    const double n = 1.0 / sqrt(fabs(gdot(G, v, v)));
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= n;
}

__device__ __forceinline__ void t_project_out(double va[4], const double vb[4], const Gcov &G) {
    const double f = gdot(G, va, vb) / gdot(G, vb, vb);
#pragma unroll
    for (int i = 0; i < 4; ++i) va[i] -= vb[i] * f;
}

/* make_tetrad (tetrads.cpp:68-124): Gram-Schmidt of (u, trial, e2, e3) in g; returns e_con only,
 * e_cov rows are lower(e_con) with row 0 negated and are formed on demand. */
__device__ __forceinline__ void make_tetrad(const double u_con[4], double trial[4], const Gcov &G, double ec[4][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ec[0][i] = u_con[i];
    t_normalize(ec[0], G);
    if (gdot(G, trial, trial) < 1.0e-30) {
#pragma unroll
        for (int i = 0; i < 4; ++i) trial[i] = (i == 1) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) ec[1][i] = trial[i];
    t_project_out(ec[1], ec[0], G);
    t_normalize(ec[1], G);
#pragma unroll
    for (int i = 0; i < 4; ++i) ec[2][i] = (i == 2) ? 1.0 : 0.0;
    t_project_out(ec[2], ec[0], G);
    t_project_out(ec[2], ec[1], G);
    t_normalize(ec[2], G);
#pragma unroll
    for (int i = 0; i < 4; ++i) ec[3][i] = (i == 3) ? 1.0 : 0.0;
    t_project_out(ec[3], ec[0], G);
    t_project_out(ec[3], ec[1], G);
    t_project_out(ec[3], ec[2], G);
    t_normalize(ec[3], G);
}

/* row i of e_cov = lower(e_con[i]) (row 0 negated) */
__device__ __forceinline__ void tetrad_cov_row(const double ec[4][4], const Gcov &G, int i, double el[4]) {
    lower(G, ec[i], el);
    if (i == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) el[j] = -el[j];
    }
}

__device__ __forceinline__ void boost(const double v[4], const double u[4], double vp[4]) {
    const double g = u[0];
    const double v_ = sqrt(fabs(1.0 - 1.0 / (g * g)));
    const double ig = 1.0 / (g * v_ + EPS);
    const double n1 = u[1] * ig, n2 = u[2] * ig, n3 = u[3] * ig;
    const double gm1 = g - 1.0;
    vp[0] = u[0] * v[0] - u[1] * v[1] - u[2] * v[2] - u[3] * v[3];
    vp[1] = -u[1] * v[0] + (1.0 + n1 * n1 * gm1) * v[1] + n1 * n2 * gm1 * v[2] + n1 * n3 * gm1 * v[3];
    vp[2] = -u[2] * v[0] + n2 * n1 * gm1 * v[1] + (1.0 + n2 * n2 * gm1) * v[2] + n2 * n3 * gm1 * v[3];
    vp[3] = -u[3] * v[0] + n3 * n1 * gm1 * v[1] + n3 * n2 * gm1 * v[2] + (1.0 + n3 * n3 * gm1) * v[3];
}

__device__ __forceinline__ void sample_rand_dir(Rng &g, double &x, double &y, double &z) {
    z = uniform(g) * 2.0 - 1.0;
    double s, c;
    fsincospi(2.0 * uniform(g), s, c); /* phi = 2 pi u: exact reduction */
    const double sq = sqrt(1.0 - z * z);
    x = sq * c;
    y = sq * s;
}

__device__ __forceinline__ double sample_y_distr(Rng &g, double theta_e) {
    double pi_3 = sqrt(kPi) / 4.0;
    double pi_4 = sqrt(0.5 * theta_e) / 2.0;
    double pi_5 = 3.0 * sqrt(kPi) * theta_e / 8.0;
    double pi_6 = theta_e * sqrt(0.5 * theta_e);
    const double s_3 = pi_3 + pi_4 + pi_5 + pi_6;
    pi_3 /= s_3;
    pi_4 /= s_3;
    pi_5 /= s_3;
    double y, x2, prob;
    do {
        const double x1 = uniform(g);
        int dof;
        if (x1 < pi_3)
            dof = 3;
        else if (x1 < pi_3 + pi_4)
            dof = 4;
        else if (x1 < pi_3 + pi_4 + pi_5)
            dof = 5;
        else
            dof = 6;
        const double x = chi_sq(g, dof);
        y = sqrt(x / 2.0);
        x2 = uniform(g);
        const double num = sqrt(1.0 + 0.5 * theta_e * y * y);
        const double den = (1.0 + y * sqrt(0.5 * theta_e));
        prob = num / den;
    } while (x2 >= prob);
    return y;
}

__device__ __forceinline__ void sample_electron(Rng &g, const double k[4], double p[4], double theta_e) {
    double sigma_kn, gamma_e, beta_e, mu, x1;
    do {
        const double y = sample_y_distr(g, theta_e);
        gamma_e = y * y * theta_e + 1.0;
        beta_e = sqrt(1.0 - 1.0 / (gamma_e * gamma_e));
        const double u = uniform(g);
        const double det = 1.0 + 2.0 * beta_e + beta_e * beta_e - 4.0 * beta_e * u;
        mu = (1.0 - sqrt(det)) / beta_e;
        mu = fmin(fmax(mu, -1.0), 1.0);
        const double k_ = gamma_e * (1.0 - beta_e * mu) * k[0];
        if (k_ < 1.0e-3)
            sigma_kn = 1.0 - 2.0 * k_;
        else
            sigma_kn = (3.0 / (4.0 * k_ * k_)) * (2.0 + k_ * k_ * (1.0 + k_) / ((1.0 + 2.0 * k_) * (1.0 + 2.0 * k_)) +
                                                  (k_ * k_ - 2.0 * k_ - 2.0) / (2.0 * k_) * flog(1.0 + 2.0 * k_));
        x1 = uniform(g);
    } while (x1 >= sigma_kn);
    const double iv0 = 1.0 / sqrt(k[1] * k[1] + k[2] * k[2] + k[3] * k[3]);
    const double v0x = k[1] * iv0, v0y = k[2] * iv0, v0z = k[3] * iv0;
    double n0x, n0y, n0z;
    sample_rand_dir(g, n0x, n0y, n0z);
    const double n0dotv0 = v0x * n0x + v0y * n0y + v0z * n0z;
    double v1x = n0x - n0dotv0 * v0x, v1y = n0y - n0dotv0 * v0y, v1z = n0z - n0dotv0 * v0z;
    const double iv1 = 1.0 / sqrt(v1x * v1x + v1y * v1y + v1z * v1z);
    v1x *= iv1;
    v1y *= iv1;
    v1z *= iv1;
    const double v2x = v0y * v1z - v0z * v1y, v2y = v0z * v1x - v0x * v1z, v2z = v0x * v1y - v0y * v1x;
    double s_phi, c_phi;
    fsincospi(2.0 * uniform(g), s_phi, c_phi); /* phi = 2 pi u */
    const double c_th = mu, s_th = sqrt(1. - mu * mu);
    const double gb = gamma_e * beta_e;
    p[0] = gamma_e;
    p[1] = gb * (c_th * v0x + s_th * (c_phi * v1x + s_phi * v2x));
    p[2] = gb * (c_th * v0y + s_th * (c_phi * v1y + s_phi * v2y));
    p[3] = gb * (c_th * v0z + s_th * (c_phi * v1z + s_phi * v2z));
}

__device__ __forceinline__ double sample_klein_nishina(Rng &g, double k0) {
    const double k0pmin = k0 / (1.0 + 2.0 * k0), k0pmax = k0;
    const double xmax = 2.0 * (1.0 + 2.0 * k0 + 2.0 * k0 * k0) / (k0 * k0 * (1.0 + 2.0 * k0));
    double x1, kt;
    while (true) {
        kt = k0pmin + (k0pmax - k0pmin) * uniform(g);
        x1 = xmax * uniform(g);
        const double ch = 1.0 + 1.0 / k0 - 1.0 / kt;
        const double kn = (k0 / kt + kt / k0 - 1.0 + ch * ch) / (k0 * k0);
        if (!(x1 >= kn)) break;
    }
    return kt;
}

__device__ __forceinline__ double sample_thomson(Rng &g) {
    double x1, x2;
    do {
        x1 = 2.0 * uniform(g) - 1.0;
        x2 = (3.0 / 4.0) * uniform(g);
    } while (x2 >= (3.0 / 8.0) * (1.0 + x1 * x1));
    return x1;
}

__device__ __forceinline__ void sample_scattered(Rng &g, const double k[4], double p[4], double kp[4]) {
    double ke[4];
    boost(k, p, ke);
    double k0p, c_th;
    if (ke[0] > 1.0e-4) {
        k0p = sample_klein_nishina(g, ke[0]);
        c_th = 1.0 - 1.0 / k0p + 1.0 / ke[0];
    } else {
        k0p = ke[0];
        c_th = sample_thomson(g);
    }
    const double s_th = sqrt(fabs(1.0 - c_th * c_th));
    const double ik = 1.0 / ke[0];
    const double v0x = ke[1] * ik, v0y = ke[2] * ik, v0z = ke[3] * ik;
    double n0x, n0y, n0z;
    sample_rand_dir(g, n0x, n0y, n0z);
    const double n0dotv0 = v0x * n0x + v0y * n0y + v0z * n0z;
    double v1x = n0x - n0dotv0 * v0x, v1y = n0y - n0dotv0 * v0y, v1z = n0z - n0dotv0 * v0z;
    const double iv1 = 1.0 / sqrt(v1x * v1x + v1y * v1y + v1z * v1z);
    v1x *= iv1;
    v1y *= iv1;
    v1z *= iv1;
    const double v2x = v0y * v1z - v0z * v1y, v2y = v0z * v1x - v0x * v1z, v2z = v0x * v1y - v0y * v1x;
    double s_phi, c_phi;
    fsincospi(2.0 * uniform(g), s_phi, c_phi); /* phi = 2 pi u */
    p[1] = -p[1];
    p[2] = -p[2];
    p[3] = -p[3];
    const double d1 = c_th * v0x + s_th * (c_phi * v1x + s_phi * v2x);
    const double d2 = c_th * v0y + s_th * (c_phi * v1y + s_phi * v2y);
    const double d3 = c_th * v0z + s_th * (c_phi * v1z + s_phi * v2z);
    const double kpe[4] = {k0p, k0p * d1, k0p * d2, k0p * d3};
    boost(kpe, p, kp);
}

} /* namespace grm */
