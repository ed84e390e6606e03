/*
 * grm_emit.hip -- superphoton emission on the GPU (gfx950): the zone walk and sampler of the
 * reference's make_super_photon path (m-torhan/cuda-grmonty harm_model.cpp:673-811; init_zone
 * :1337-1389; jnu_mixed.cpp:75-125), feeding the transport kernel without a host round trip.
 *
 * The reference emits on 5 host threads (harm_model.cpp:842-892) while one mt19937 stream per
 * worker makes the photon list depend on thread timing.  Here the list depends only on the seed:
 *
 *   zone_count_scan  (one workgroup)  count_z = floor(nz) + (frac(nz) > u_z), u_z = first draw of
 *                                     the zone stream (:693-697); exclusive scan -> offsets
 *   emit_kernel      (one lane per photon)  zone by binary search of the offsets; photon p of zone
 *                                     z draws from its own Philox stream (counter words
 *                                     (draw, p + 1, z, 'EMIT' ^ z_hi)), so lanes never wait on
 *                                     each other; rejection sampling of nu (f_eval / weight) and
 *                                     of the emission angle (synch), tetrad -> coordinate frame
 *                                     (sample_zone_photon :706-782)
 *
 * The per-zone fluid state, tetrad, nz and dn_max come from the host zone table
 * (grm_model_zone_table), so host and device emission start from identical bits; the host
 * emitter (grm_model_emit) uses the same streams, and so does the oracle's Philox emission mode.
 * HBM traffic: 272 B zone record (L2-resident, shared by the zone's photons) in, 128 B photon out.
 */
#include <hip/hip_runtime.h>

#include <string>

#include "grm_device.h"
#include "grm_emit.h"

using namespace grm;

namespace {

constexpr int SCAN_THREADS = 1024;
constexpr int EMIT_BLOCK = 256;
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

__device__ __forceinline__ uint32_t zone_count(const grm_emit_zone *zones, uint64_t z, uint32_t k0, uint32_t k1) {
    const double nz = zones[z].nz;
    Rng r = zone_rng(k0, k1, z, 0);
    const double u = uniform(r);
    return (fmod(nz, 1.0) > u) ? (uint32_t)((int)nz + 1) : (uint32_t)(int)nz;
}

/* counts of zones z0 + q * stride, q in [0, n), and their exclusive prefix sum off[0..n] (one
 * workgroup; each thread owns a contiguous chunk and recomputes its counts in the second pass
 * instead of storing) */
__global__ __launch_bounds__(SCAN_THREADS) void zone_count_scan(const grm_emit_zone *zones, uint64_t z0, uint64_t stride,
                                                                uint64_t n, uint32_t k0, uint32_t k1, unsigned long long *off,
                                                                unsigned long long *h_total) {
    __shared__ unsigned long long part[SCAN_THREADS];
    const uint64_t per = (n + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint64_t a = min(n, (uint64_t)threadIdx.x * per), b = min(n, a + per);
    unsigned long long s = 0;
    for (uint64_t q = a; q < b; ++q) s += zone_count(zones, z0 + q * stride, k0, k1);
    part[threadIdx.x] = s;
    __syncthreads();
    /* Hillis-Steele inclusive scan of the 1024 chunk sums */
    for (int d = 1; d < SCAN_THREADS; d <<= 1) {
        const unsigned long long v = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0ull;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned long long run = part[threadIdx.x] - s;
    for (uint64_t q = a; q < b; ++q) {
        off[q] = run;
        run += zone_count(zones, z0 + q * stride, k0, k1);
    }
    if (threadIdx.x == SCAN_THREADS - 1) {
        off[n] = part[SCAN_THREADS - 1];
        *h_total = part[SCAN_THREADS - 1]; /* host-mapped: no read-back copy */
        __threadfence_system();
    }
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
__device__ void sample_photon(const Params &P, const EmitParams &E, const grm_emit_zone &Z, Rng &r,
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

__global__ __launch_bounds__(EMIT_BLOCK) void emit_kernel(Params P, EmitParams E, uint64_t z0, uint64_t stride,
                                                          uint64_t n_zones, const unsigned long long *off,
                                                          uint64_t total, grm_init_photon *out) {
    const uint64_t g = (uint64_t)blockIdx.x * EMIT_BLOCK + threadIdx.x;
    if (g >= total) return;
    /* zone q with off[q] <= g < off[q + 1] (empty zones have off[q] == off[q + 1]) */
    uint64_t lo = 0, hi = n_zones; /* invariant: off[lo] <= g < off[hi] */
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (off[mid] <= g)
            lo = mid;
        else
            hi = mid;
    }
    const uint64_t z = z0 + lo * stride;
    const grm_emit_zone &Z = E.zones[z];
    Rng r = zone_rng(E.k0, E.k1, z, g - off[lo] + 1);
    grm_init_photon ph;
    sample_photon(P, E, Z, r, ph);
    /* 8 x 16-B stores */
    const double2 *s = reinterpret_cast<const double2 *>(&ph);
    double2 *d = reinterpret_cast<double2 *>(out + g);
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = s[q];
}

} /* namespace */

int grm_emit_launch(const Params &P, const EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                    unsigned long long *d_off,
                    hipStream_t s, unsigned long long *h_total, grm_init_photon **out, size_t *out_cap, uint64_t *n_out,
                    std::string &err) {
    auto chk = [&](hipError_t st, const char *what) {
        if (st == hipSuccess) return true;
        err = std::string(what) + ": " + hipGetErrorString(st);
        return false;
    };
    *n_out = 0;
    if (n_zones == 0) return 0;
    /* h_total: a host-mapped word the scan kernel writes itself (no copy kernel on the stream) */
    hipLaunchKernelGGL(zone_count_scan, dim3(1), dim3(SCAN_THREADS), 0, s, E.zones, z0, stride, n_zones, E.k0, E.k1,
                       d_off, h_total);
    if (!chk(hipGetLastError(), "zone_count_scan") || !chk(hipStreamSynchronize(s), "sync")) return -1;
    const unsigned long long total = *(volatile unsigned long long *)h_total;
    if (total > *out_cap) {
        /* grown with 1/8 headroom: the count moves by ~0.1 % from seed to seed, and an exact fit
         * reallocated whenever a pass drew more photons than every pass before -- hipFree waits
         * for the whole device, so one engine's emission then waited for every other stream's
         * work (the emulated ranks sharing a GPU started up to 0.5 s late, profiles/r04v_phases_w8.log),
         * and a bench pass paid the free + malloc of ~2 GB in its timed region */
        if (*out) (void)hipFree(*out);
        *out = nullptr;
        *out_cap = 0;
        const unsigned long long cap = total + total / 8;
        if (!chk(hipMalloc(out, cap * sizeof(grm_init_photon)), "emit buffer")) return -1;
        *out_cap = cap;
    }
    if (total > 0) {
        const uint64_t blocks = (total + EMIT_BLOCK - 1) / EMIT_BLOCK;
        if (blocks > 0xFFFFFFFFull) {
            err = "emit: too many photons for one launch";
            return -1;
        }
        hipLaunchKernelGGL(emit_kernel, dim3((unsigned)blocks), dim3(EMIT_BLOCK), 0, s, P, E, z0, stride, n_zones,
                           d_off, (uint64_t)total, *out);
        if (!chk(hipGetLastError(), "emit_kernel") || !chk(hipStreamSynchronize(s), "emit sync")) return -1;
    }
    *n_out = total;
    return 0;
}
