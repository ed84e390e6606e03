/*
 * grmonty_amd_debug.h -- diagnostic and test entry points of libgrmonty_amd.so.
 *
 * Not part of the drop-in boundary (include/grmonty_amd.h, which replaces the reference's
 * cuda_super_photon namespace, super_photon.cuh:15-63): these read the engine's internal records
 * (per-wave timing of a -DGRM_TIMING build, the watchdog's abandoned photons, raw device counters,
 * the live-bias warm-up's admission log) or evaluate one device function per input (the
 * per-function parity probes of tests/test_gpu_probes.py).  Tools and tests use them; a host
 * integrating the engine needs none.
 */
#ifndef GRMONTY_AMD_DEBUG_H
#define GRMONTY_AMD_DEBUG_H

#include "grmonty_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* diagnostic: per-region wave cycles of a -DGRM_TIMING build, 48 slots (returns 1 if the build
 * is instrumented, 0 if not; out[] then stays zero) */
int grm_engine_debug_timing(grm_engine *e, uint64_t out[48], int reset);

/* diagnostic: per-wave record of the last transport launch, 4 x u64 per wave: start and exit
 * (s_memrealtime, 100 MHz), loop trips, superphotons tracked.  out holds cap waves; returns the
 * number of waves of the grid (-1 before the first launch). */
int64_t grm_engine_debug_waves(grm_engine *e, uint64_t *out, size_t cap);

/* diagnostic: state of the photons the watchdog abandoned, 16 doubles each: id, n_step, phase, depth,
 * pend, w, e_0_s, dl, x[4], k[4].  out holds cap records; returns the records kept (<= 256). */
int64_t grm_engine_debug_stuck(grm_engine *e, double *out, size_t cap);
/* raw device counters: n_recorded, n_scatt, max_tau_scatt bits, n_steps, n_tracked, n_children,
 * n_overflow, n_dropped, n_primaries, max photon steps, lives > 1e5 steps, n_abandoned, abort, n_nan,
 * waves whose kernel-argument check failed, and word 15 = the multi-rank warm-up state of the
 * pass block (photons admitted << 32, plus the photons in flight as a signed low word, plus bit 63
 * once this rank's admission is over and bit 62 once this rank's launch of the pass has started --
 * the job's start barrier, GRM_OPT_JOB_START_WAIT_MS; 0 on a single GPU) */
int grm_engine_debug_counters(grm_engine *e, uint64_t out[16]);
/* diagnostic: the phases of the last call's main launch, s_memrealtime ticks (100 MHz): first wave
 * start, end of the live-bias warm-up admission (0 = none), the pool's last claim chunk taken (0 =
 * not reached), last wave exit */
int grm_engine_debug_phases(grm_engine *e, uint64_t out[4]);
/* the live-bias warm-up's admission log of the same launch: out[2i] = s_memrealtime tick when batch
 * i + 1 opened, out[2i + 1] = photons in flight then (i < cap); returns the number of openings */
int64_t grm_engine_debug_admissions(grm_engine *e, uint64_t *out, size_t cap);

/* --- experiment: the role-split bulk kernel (csrc/grm_split.hip) ---------- */
/* Measured 12 % slower than track_kernel and not in the product library: only a variant build
 * (VFLAGS=-DGRM_WITH_SPLIT tools/build_variant.sh split) accepts these options; the product's
 * grm_engine_set_option rejects them. */
enum {
    /* the bulk transport kernel: 0 = track_kernel, 1 = split_kernel (waves 0-3 geometry, 4-7
     * interaction), 2 = split_kernel with the roles dealt by SIMD */
    GRM_OPT_SPLIT = 23,
    /* an interaction wave evaluates its ready steps once this many 64ths of its active lanes have
     * one (default 48), or after GRM_OPT_SPLIT_SPIN short sleeps (default 4) */
    GRM_OPT_SPLIT_THR = 24,
    GRM_OPT_SPLIT_SPIN = 25,
    /* a geometry wave makes its push attempts once this many 64ths of its live lanes can (default 24) */
    GRM_OPT_SPLIT_GTHR = 26,
    /* consecutive ready slots an interaction lane evaluates per round (1..3, default 1) */
    GRM_OPT_SPLIT_BATCH = 27
};

/* --- per-function device probes (parity tests; one lane per input) --------------------- */
/* which: see GRM_PROBE_* in DESIGN.md / csrc/grm_probe.hip. in/out are host arrays of
 * n * in_stride / n * out_stride doubles. */
int grm_probe(grm_engine *e, int which, const double *in, int in_stride, double *out, int out_stride, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* GRMONTY_AMD_DEBUG_H */
