/*
 * grm_emit.h -- kernel-argument block and launcher of the device emission (grm_emit.hip),
 * shared with the engine's C-ABI entry points (grm_engine.hip).
 */
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "grm_device.h"

namespace grm {

/* uniform across lanes: tables + derived constants of sample_zone_photon (harm_model.cpp:706-792)
 * and jnu_mixed::f_eval (jnu_mixed.cpp:113-125), host libm values (consts.hpp) */
struct EmitParams {
    const grm_emit_zone *zones; /* all n1*n2 zones */
    const double *weight;       /* [201] log weight */
    const double *f;            /* [201] log F */
    double l_nu_min, n_l_n, d_l_nu;
    double jnu_l_min_k, jnu_d_l_k;
    uint32_t k0, k1;            /* Philox key = seed */
};

} /* namespace grm */


/* ---- the per-photon sampler, shared by emit_kernel (grm_emit.hip) and the transport kernel's
 * in-launch emission (grm_engine.hip, grm_engine_emit_track) ---- */
namespace grm {

constexpr uint32_t EMIT_SALT = 0x454D4954u; /* 'EMIT' */
constexpr double JNU_MIN_K = 0.002, JNU_MAX_K = 1.0e7;
constexpr double JNU_K_FAC = 9 * kPi * ME * CL / EE;

/* stream of zone z; slot 0 is the count draw, photon p of the zone uses slot p + 1 */
__device__ __forceinline__ Rng zone_rng(uint32_t k0, uint32_t k1, uint64_t z, uint64_t slot) {
    Rng r;
    r.k0 = k0;
    r.k1 = k1;
    r.id = ((uint64_t)(EMIT_SALT ^ (uint32_t)(z >> 32)) << 32) | (uint32_t)z;
    r.ctr = 0;
    r.ctr_hi = (uint32_t)slot;
    return r;
}

/* linear_interp_weight (harm_model.cpp:784-792); u = 1 exactly gives nu = nu_max: stay in the table */
__device__ __forceinline__ double interp_weight(const EmitParams &E, double nu) {
    double d = (log(nu) - E.l_nu_min) / E.d_l_nu;
    const int i = min((int)d, GRM_N_E_SAMP - 1);
    d -= i;
    return exp((1.0 - d) * E.weight[i] + d * E.weight[i + 1]);
}

/* jnu_mixed::f_eval (jnu_mixed.cpp:113-125, linear_interp_f :160-167) */
__device__ __forceinline__ double f_eval(const EmitParams &E, double theta_e, double b, double nu) {
    const double k = JNU_K_FAC * nu / (b * theta_e * theta_e);
    if (k > JNU_MAX_K) return 0.0;
    if (k < JNU_MIN_K) {
        const double x = pow(k, 1.0 / 3.0);
        return x * (37.67503800178 + 2.240274341836 * x);
    }
    double d = (log(k) - E.jnu_l_min_k) / E.jnu_d_l_k;
    const int i = min((int)d, GRM_N_E_SAMP - 1);
    d -= i;
    return exp((1.0 - d) * E.f[i] + d * E.f[i + 1]);
}

/* sample_zone_photon (harm_model.cpp:706-782) from the photon's own stream */
__device__ __forceinline__ void sample_photon(const Params &P, const EmitParams &E, const grm_emit_zone &Z, Rng &r,
                              grm_init_photon &ph) {
    double nu, w;
    do {
        nu = exp(uniform(r) * E.n_l_n + E.l_nu_min);
        w = interp_weight(E, nu);
    } while (uniform(r) > (f_eval(E, Z.theta_e, Z.b, nu) / (w + 1.0e-100)) / Z.dn_max);
    const double ln_te = log(Z.theta_e);
    const double j_max = synch_s(P, nu, Z.n_e, Z.theta_e, Z.b, 1.0, ln_te); /* sin(pi/2) = 1 */
    double cos_th, th;
    do {
        cos_th = 2.0 * uniform(r) - 1.0;
        th = acos(cos_th);
    } while (uniform(r) > synch_s(P, nu, Z.n_e, Z.theta_e, Z.b, sin(th), ln_te) / j_max);
    const double sin_th = sqrt(1.0 - cos_th * cos_th);
    const double phi = 2.0 * kPi * uniform(r);
    const double cos_phi = cos(phi), sin_phi = sin(phi);
    const double e = nu * HPL / (ME * CL * CL);
    const double kt[4] = {e, e * cos_th, e * sin_th * cos_phi, e * sin_th * sin_phi};
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        double s = 0.0;
#pragma unroll
        for (int b = 0; b < 4; ++b) s += Z.e_con[b][a] * kt[b];
        ph.k[a] = s;
    }
    /* tetrad_to_coordinate(e_cov, (-k0, k1, k2, k3)): components 0 and 3 only */
    double t0 = 0.0, t3 = 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const double kb = b == 0 ? -kt[0] : kt[b];
        t0 += Z.e_cov_t[b] * kb;
        t3 += Z.e_cov_z[b] * kb;
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) ph.x[a] = Z.x[a];
    ph.w = w;
    ph.e = -t0;
    ph.e_0 = -t0;
    ph.l = t3;
    ph.n_e_0 = Z.n_e;
    ph.theta_e_0 = Z.theta_e;
    ph.b_0 = Z.b;
    ph.n_scatt = 0;
    ph.pad_ = 0;
}


/* photon g of the emitted batch: its zone q (off[q] <= g < off[q + 1]; empty zones have off[q] ==
 * off[q + 1]) by binary search, its own Philox stream (slot g - off[q] + 1 of the zone's), the
 * sampler, eight 16-B stores */
template <bool NT = false> /* NT: non-temporal stores (the batch streams past L2, whose working set is the transport's) */
__device__ __forceinline__ void emit_photon(const Params &P, const EmitParams &E, uint64_t z0, uint64_t stride,
                                            uint64_t n_zones, const unsigned long long *off, uint64_t g,
                                            grm_init_photon *out) {
    uint64_t lo = 0, hi = n_zones; /* invariant: off[lo] <= g < off[hi] */
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (off[mid] <= g)
            lo = mid;
        else
            hi = mid;
    }
    const uint64_t z = z0 + lo * stride;
    Rng r = zone_rng(E.k0, E.k1, z, g - off[lo] + 1);
    grm_init_photon ph;
    sample_photon(P, E, E.zones[z], r, ph);
    typedef double v2d __attribute__((ext_vector_type(2)));
    const v2d *s = reinterpret_cast<const v2d *>(&ph);
    v2d *d = reinterpret_cast<v2d *>(out + g);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (NT)
            __builtin_nontemporal_store(s[q], d + q);
        else
            d[q] = s[q];
    }
}

} /* namespace grm */

/* zone counts + scan of zones z0 + q * stride, q in [0, n_zones), then one lane per photon into
 * *out (grown to fit; *out_cap updated); d_off holds n_zones + 1 offsets.  Synchronous; 0 = OK. */
int grm_emit_launch(const grm::Params &P, const grm::EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                    unsigned long long *d_off, hipStream_t s, unsigned long long *h_total, grm_init_photon **out,
                    size_t *out_cap, uint64_t *n_out, std::string &err);
/* its two halves: the counts and scan (synchronous: the total sizes *out) ... */
int grm_emit_count(const grm::EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones, unsigned long long *d_off,
                   hipStream_t s, unsigned long long *h_total, grm_init_photon **out, size_t *out_cap, uint64_t *n_out,
                   std::string &err);
/* ... and the photons, queued on s */
int grm_emit_fill(const grm::Params &P, const grm::EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                  const unsigned long long *d_off, uint64_t total, grm_init_photon *out, hipStream_t s, std::string &err);
/* only the photons at claim positions [0, n_pos) (position q: photon (q mod 2^sh) m + q / 2^sh), queued on s */
int grm_emit_positions(const grm::Params &P, const grm::EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                       const unsigned long long *d_off, uint64_t total, grm_init_photon *out, int sh, uint64_t m,
                       uint64_t n_pos, hipStream_t s, std::string &err);
