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

__global__ __launch_bounds__(EMIT_BLOCK) void emit_kernel(Params P, EmitParams E, uint64_t z0, uint64_t stride,
                                                          uint64_t n_zones, const unsigned long long *off,
                                                          uint64_t total, grm_init_photon *out) {
    const uint64_t g = (uint64_t)blockIdx.x * EMIT_BLOCK + threadIdx.x;
    if (g < total) emit_photon(P, E, z0, stride, n_zones, off, g, out);
}

/* the photons at claim positions [0, n_pos) of the transport's interleaved claim order (position q is
 * photon (q mod 2^sh) m + q / 2^sh; holes past `total` skipped): the live-bias warm-up's admission
 * batches, emitted ahead of a transport launch that emits the rest itself (grm_engine_emit_track) */
__global__ __launch_bounds__(EMIT_BLOCK) void emit_pos_kernel(Params P, EmitParams E, uint64_t z0, uint64_t stride,
                                                              uint64_t n_zones, const unsigned long long *off,
                                                              uint64_t total, grm_init_photon *out, int sh, uint64_t m,
                                                              uint64_t n_pos) {
    const uint64_t q = (uint64_t)blockIdx.x * EMIT_BLOCK + threadIdx.x;
    if (q >= n_pos) return;
    const uint64_t g = (q & ((1ull << sh) - 1)) * m + (q >> sh);
    if (g < total) emit_photon(P, E, z0, stride, n_zones, off, g, out);
}

} /* namespace */

namespace {
bool emit_chk(hipError_t st, const char *what, std::string &err) {
    if (st == hipSuccess) return true;
    err = std::string(what) + ": " + hipGetErrorString(st);
    return false;
}
} /* namespace */

int grm_emit_count(const EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones, unsigned long long *d_off,
                   hipStream_t s, unsigned long long *h_total, grm_init_photon **out, size_t *out_cap, uint64_t *n_out,
                   std::string &err) {
    *n_out = 0;
    if (n_zones == 0) return 0;
    /* h_total: a host-mapped word the scan kernel writes itself (no copy kernel on the stream) */
    hipLaunchKernelGGL(zone_count_scan, dim3(1), dim3(SCAN_THREADS), 0, s, E.zones, z0, stride, n_zones, E.k0, E.k1,
                       d_off, h_total);
    if (!emit_chk(hipGetLastError(), "zone_count_scan", err) || !emit_chk(hipStreamSynchronize(s), "sync", err))
        return -1;
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
        if (!emit_chk(hipMalloc(out, cap * sizeof(grm_init_photon)), "emit buffer", err)) return -1;
        *out_cap = cap;
    }
    *n_out = total;
    return 0;
}

int grm_emit_fill(const Params &P, const EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                  const unsigned long long *d_off, uint64_t total, grm_init_photon *out, hipStream_t s,
                  std::string &err) {
    if (total == 0) return 0;
    const uint64_t blocks = (total + EMIT_BLOCK - 1) / EMIT_BLOCK;
    if (blocks > 0xFFFFFFFFull) {
        err = "emit: too many photons for one launch";
        return -1;
    }
    hipLaunchKernelGGL(emit_kernel, dim3((unsigned)blocks), dim3(EMIT_BLOCK), 0, s, P, E, z0, stride, n_zones, d_off,
                       total, out);
    return emit_chk(hipGetLastError(), "emit_kernel", err) ? 0 : -1;
}

int grm_emit_positions(const Params &P, const EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                       const unsigned long long *d_off, uint64_t total, grm_init_photon *out, int sh, uint64_t m,
                       uint64_t n_pos, hipStream_t s, std::string &err) {
    if (n_pos == 0 || total == 0) return 0;
    const uint64_t blocks = (n_pos + EMIT_BLOCK - 1) / EMIT_BLOCK;
    hipLaunchKernelGGL(emit_pos_kernel, dim3((unsigned)blocks), dim3(EMIT_BLOCK), 0, s, P, E, z0, stride, n_zones,
                       d_off, total, out, sh, m, n_pos);
    return emit_chk(hipGetLastError(), "emit_pos_kernel", err) ? 0 : -1;
}

int grm_emit_launch(const Params &P, const EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                    unsigned long long *d_off, hipStream_t s, unsigned long long *h_total, grm_init_photon **out,
                    size_t *out_cap, uint64_t *n_out, std::string &err) {
    if (grm_emit_count(E, z0, stride, n_zones, d_off, s, h_total, out, out_cap, n_out, err)) return -1;
    if (grm_emit_fill(P, E, z0, stride, n_zones, d_off, *n_out, *out, s, err)) return -1;
    return emit_chk(hipStreamSynchronize(s), "emit sync", err) ? 0 : -1;
}
