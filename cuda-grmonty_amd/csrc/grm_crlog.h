/*
 * grm_crlog.h -- a correctly rounded log and glibc's log10 construction, for the device table
 * builders (csrc/grm_tables.hip) whose entries must come out as the host builders' do.
 *
 * The host builds its tables with glibc (hotcross.cpp:144-151 evaluates log(1 + 2w) inside the
 * Klein-Nishina expression, which cancels ~6 digits just above its w = 1e-3 switch, so a last-bit
 * difference of that log is ~1e-10 of sigma).  glibc's log is correctly rounded but for inputs
 * within ~0.005 ulp of a rounding boundary (0.02 % of random arguments); ocml's is not.  cr_log
 * takes ocml's log y0 and adds log(x e^-y0), computed from a double-double e^y0, so its one
 * rounding is the correctly rounded log.  glibc's log10 is fdlibm's e_log10 construction,
 * k log10(2) split in two parts plus log(m) / ln 10 of the mantissa; grm_log10 is that construction
 * on cr_log.  tests/native/crlog_check.cpp compiles this header on the host and checks both against
 * glibc.
 *
 * The includer defines GRM_CR_FN (function qualifiers) and GRM_CR_LOG (the libm-grade log the
 * correction starts from); fma / rint / ldexp are the C math functions of both compilers.
 */
#ifndef GRM_CRLOG_H
#define GRM_CRLOG_H

#include <stdint.h>


namespace grm_cr {

struct DD {
    double h, l;
};

GRM_CR_FN DD two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
GRM_CR_FN DD quick_two_sum(double a, double b) {
    const double s = a + b;
    return {s, b - (s - a)};
}
GRM_CR_FN DD dd_mul(DD a, DD b) {
    const double p = a.h * b.h;
    const double e = fma(a.h, b.h, -p) + (a.h * b.l + a.l * b.h);
    return quick_two_sum(p, e);
}
GRM_CR_FN DD dd_add(DD a, DD b) {
    const DD s = two_sum(a.h, b.h);
    return quick_two_sum(s.h, s.l + a.l + b.l);
}
GRM_CR_FN DD dd_div_int(DD a, double n) {
    const double q1 = a.h / n;
    const double r = fma(-q1, n, a.h) + a.l;
    return quick_two_sum(q1, r / n);
}

/* e^y in double-double, |y| < 700: y = k ln 2 + t (ln 2 in two parts, the products exact by fma),
 * |t| <= ln 2 / 2, e^t by its Taylor series in nested form (t^18 / 18! < 1e-23, far below the
 * 1e-19 that the correction of an ulp-accurate log needs) */
GRM_CR_FN DD dd_exp(double y) {
    const double LN2_HI = 6.93147180559945286227e-01, LN2_LO = 2.31904681384629955842e-17;
    const double k = rint(y * 1.44269504088896338700e+00);
    const double p = k * LN2_HI, q = k * LN2_LO;
    DD t = dd_add({y, 0.0}, {-p, -fma(k, LN2_HI, -p)});
    t = dd_add(t, {-q, -fma(k, LN2_LO, -q)});
    DD s = {1.0, 0.0};
    for (int i = 17; i >= 1; --i) s = dd_add({1.0, 0.0}, dd_div_int(dd_mul(t, s), (double)i));
    return {ldexp(s.h, (int)k), ldexp(s.l, (int)k)};
}

/* log(x) for a positive normal finite x, correctly rounded (but within ~1e-30 of a boundary):
 * y0 = libm log(x), r = x e^-y0 - 1 (x - e^y0 is exact: the two agree to an ulp or two),
 * log(x) = y0 + log1p(r), |r| ~ 1e-16 */
GRM_CR_FN double cr_log(double x) {
    const double y0 = GRM_CR_LOG(x);
    const DD e = dd_exp(y0);
    const double r = ((x - e.h) - e.l) / e.h;
    return y0 + (r - 0.5 * r * r);
}

/* log10(x) for a positive normal finite x as glibc forms it (fdlibm e_log10): x = 2^k m with
 * m in [1, 2) (or [0.5, 1) when k < 0), log10(x) = (k log10_2lo + log(m) / ln 10) + k log10_2hi */
GRM_CR_FN double grm_log10(double x) {
#ifdef __clang__
#pragma clang fp contract(off) /* glibc's products and sums, each rounded (no FMA on its build) */
#endif
    const double ivln10 = 4.34294481903251816668e-01, log10_2hi = 3.01029995663611771306e-01,
                 log10_2lo = 3.69423907715893078616e-13;
    /* zero, subnormal, negative, inf and NaN arguments: the exponent rewrite below assumes a
     * positive normal number (it would give ~-308 for 0, ~308 for inf and NaN), so these take the
     * library log10 (NaN, -inf, inf as glibc) */
    if (!(x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308)) return log10(x);
    uint64_t b;
    __builtin_memcpy(&b, &x, 8);
    int32_t hx = (int32_t)(b >> 32);
    const int32_t k = (hx >> 20) - 1023;
    const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
    hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
    const double y = (double)(k + i);
    b = ((uint64_t)(uint32_t)hx << 32) | (b & 0xffffffffull);
    double m;
    __builtin_memcpy(&m, &b, 8);
    const double z = y * log10_2lo + ivln10 * cr_log(m);
    return z + y * log10_2hi;
}

} /* namespace grm_cr */

#endif
