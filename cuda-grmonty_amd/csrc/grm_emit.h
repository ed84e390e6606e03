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

/* zone counts + scan of zones z0 + q * stride, q in [0, n_zones), then one lane per photon into
 * *out (grown to fit; *out_cap updated); d_off holds n_zones + 1 offsets.  Synchronous; 0 = OK. */
int grm_emit_launch(const grm::Params &P, const grm::EmitParams &E, uint64_t z0, uint64_t stride, uint64_t n_zones,
                    unsigned long long *d_off, hipStream_t s, unsigned long long *h_total, grm_init_photon **out,
                    size_t *out_cap, uint64_t *n_out, std::string &err);
