/*
 * grmonty_amd.h -- C-ABI of the MI355X-native grmonty superphoton transport engine.
 *
 * Drop-in boundary for the reference's device boundary, namespace
 * cuda_super_photon (reference: cuda_grmonty/super_photon.cuh:15-63), plus the
 * host model API that HARMModel's callers use (harm_model.hpp / main.cpp).
 * Plain C: POD structs, pointers and sizes; no torch, no C++ types; every entry
 * point returns an int status (0 = OK) and never exits or throws across the ABI.
 *
 *   reference (CUDA build)                                 this ABI
 *   ------------------------------------------------------------------------------------
 *   cuda_super_photon::alloc_memory(header, data, units,   grm_engine_create()
 *       hotcross, f, k2)          super_photon.cuh:29-34
 *   cuda_super_photon::track_super_photons(bias_norm,      grm_engine_track() /
 *       max_tau_scatt, photon_queue, done_sem, spectrum,     grm_engine_track_device()
 *       n_rec, n_scatt)           super_photon.cuh:55-61     + grm_engine_finish()
 *   cuda_super_photon::free_memory()  super_photon.cuh:40    grm_engine_destroy()
 *   gpuErrchk -> exit()           utils.cuh:20-40          int status + grm_engine_last_error()
 *
 * The reference hands photons over through a C++ ConcurrentQueue + binary
 * semaphore (not expressible in C); here the host hands over batches of
 * InitPhoton records (photon.hpp:41-52) and scattered children stay on the
 * device (per-lane stacks + an overflow pool), never round-tripping over PCIe.
 */
#ifndef GRMONTY_AMD_H
#define GRMONTY_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GRM_N_TH_BINS 6
#define GRM_N_E_BINS 200
#define GRM_N_E_SAMP 200
#define GRM_HC_N_W 220
#define GRM_HC_N_T 80
#define GRM_NINT 20000

/* harm_data.hpp:19-44 -- HARM dump header (same field order/types as the reference) */
typedef struct grm_header {
    double t;
    int n[2];
    double x_start[4];
    double x_stop[4];
    double dx[4];
    double t_final;
    int n_step;
    double a;
    double gamma;
    double courant;
    double dt_dump;
    double dt_log;
    double dt_img;
    int dt_rdump;
    int cnt_dump;
    int cnt_img;
    int cnt_rdump;
    double dt;
    int lim;
    int failed;
    double r_in;
    double r_out;
    double h_slope;
    double r_0;
} grm_header;

/* harm_data.hpp:62-71 */
typedef struct grm_units {
    double mass_unit, l_unit, t_unit, rho_unit, u_unit, b_unit, theta_e_unit, n_e_unit;
} grm_units;

/* photon.hpp:41-52 -- emitted superphoton (15 doubles + int), 128 B */
typedef struct grm_init_photon {
    double x[4];
    double k[4];
    double w, e, l, n_e_0, theta_e_0, b_0, e_0;
    int n_scatt;
    int pad_;
} grm_init_photon;

/* harm_data.hpp:129-143 -- one (theta, energy) spectrum cell, reference field order */
typedef struct grm_spectrum_cell {
    double dn_dle, de_dle, nph, nscatt, x1i_av, x2i_sq, x3f_sq, tau_abs, tau_scatt, ne_0, theta_e_0, b_0, e_0;
} grm_spectrum_cell;

/* end-of-life record of one tracked superphoton (debug / parity traces) */
typedef struct grm_trace {
    uint64_t id;
    uint64_t parent_id;
    double w, e, x1, x2, x3, tau_abs, tau_scatt;
    int32_t n_scatt;
    int32_t n_step;
    int32_t end_reason; /* 0 recorded, 1 escaped-unbinned, 2 absorbed/horizon/roulette, 3 max-step, 4 invalid */
    int32_t ix2;
    int32_t i_e;
    int32_t pad_;
} grm_trace;

typedef struct grm_stats {
    uint64_t n_tracked;        /* superphotons tracked (primaries + scattered children) */
    uint64_t n_primaries;      /* emitted photons consumed (the reference's "created") */
    uint64_t n_children;       /* scattered children spawned on device */
    uint64_t n_steps;          /* transport loop iterations (geodesic pushes), reference n_step unit */
    uint64_t n_overflow;       /* children that spilled from lane stacks to the overflow pool */
    uint64_t n_dropped;        /* children lost to a full overflow pool (must be 0) */
    uint64_t n_launches;       /* transport kernel launches */
    double kernel_ms;          /* summed transport-kernel time (HIP events on the engine stream) */
    double last_kernel_ms;     /* duration of the most recent transport call's kernels */
    uint64_t last_steps;       /* steps in the most recent transport call */
    double last_emit_ms;       /* duration of the most recent grm_engine_emit (count + scan + sampling) */
    double max_launch_ms;      /* longest transport launch of the most recent transport call ... */
    uint64_t max_launch_steps; /* ... and the transport steps it made (per-launch roofline) */
    uint64_t max_photon_steps; /* longest superphoton life (n_step) since the last reset */
    uint64_t n_long_photons;   /* superphotons that lived more than 100k steps since the last reset */
    uint64_t n_abandoned;      /* photons dropped by the launch watchdog (GRM_OPT_WATCHDOG_MS); 0 in a good run */
    uint64_t n_nan_photons;    /* superphotons ended at a NaN position since the last reset (see grm_engine.hip) */
    uint64_t n_lone;           /* photons handed over to the lone-photon kernel since the last reset */
    double lone_ms;            /* time in lone-photon kernel launches since the last reset */
    uint64_t n_early;          /* long photons handed to the concurrent early worker since the last reset */
    double early_ms;           /* the early worker's longest launch (its stream's events) since the last reset */
    uint64_t last_grid;        /* workgroups of the most recent transport call's launch (GRM_OPT_FLIGHT_RATIO) */
    uint64_t n_early_children; /* scattered children the early worker tracked itself (GRM_OPT_EARLY_CHILDREN) */
    uint64_t n_lone_children;  /* scattered children the lone kernel tracked itself (GRM_OPT_EARLY_CHILDREN) */
} grm_stats;

typedef struct grm_engine grm_engine;

/* Engine options (grm_engine_set_option) */
enum {
    GRM_OPT_SEED = 0,        /* Philox key for transport RNG streams (default 123, consts.hpp:14) */
    GRM_OPT_BIAS_MODE = 1,   /* 0 live device counters (default, reference-like adaptive bias), 1 frozen */
    GRM_OPT_TRACE_CAP = 2,   /* >0 enables per-photon trace buffer with this capacity */
    GRM_OPT_GRID_BLOCKS = 3, /* persistent grid size override (0 = auto) */
    GRM_OPT_ID_BASE = 4,     /* first photon stream id of the next track call */
    /* frozen-bias snapshot (used when GRM_OPT_BIAS_MODE = 1; default: counters at call start) */
    GRM_OPT_FROZEN_SCATT = 5,  /* N_scatt */
    GRM_OPT_FROZEN_REC = 6,    /* N_recorded */
    GRM_OPT_FROZEN_MAXTAU = 7, /* max tau_scatt, IEEE-754 bit pattern of the double */
    /* live-bias warm-up: until this many photons have been claimed since the last reset, they are
     * admitted in batches that double the history each time (the next batch once all but a
     * 2^-GRM_OPT_WARMUP_SLACK fraction of the history has ended), so the adaptive-bias counters
     * evolve as in the serial reference (default -2 = auto: one persistent grid's worth of lanes for
     * a call of fewer than 32 x lanes photons, else 4096; -1 = lanes; 0 = off; n = n photons).
     * Tuned by the reference-semantics counters at 192^2: 0 doubles the recorded /
     * scattered counts; at photon_n = 1e5, 4096 leaves them +6 %, a grid's worth +2 %; each
     * doubling costs a batch barrier (~5-10 ms) per pass */
    GRM_OPT_WARMUP = 8,
    /* idle lanes a wavefront gathers before it takes emitted photons (1..64, default 2) */
    GRM_OPT_REFILL_MIN = 9,
    /* per-launch watchdog in ms (default 60000, 0 = off): a transport launch running longer abandons
     * its photons and exits, and the track call fails with the reason in grm_engine_error -- no input
     * can keep the GPU busy without bound (a photon's life is bounded only by 1.28M steps x 255
     * halving attempts) */
    GRM_OPT_WATCHDOG_MS = 10,
    /* scattered children a wavefront samples together (1..64, default 8): larger = less divergent
     * scattering sampling, more idle lane-trips while a batch gathers */
    GRM_OPT_CHILD_MIN = 11,
    /* warm-up straggler tolerance, log2: the next admission batch starts once at most 1/2^slack of
     * the history is still in flight (default -1 = auto: 4 for the small-pass ramp to a grid of
     * lanes and for a multi-rank job's warm-up (grm_engine_set_peers / grm_engine_link_peers), 1 for
     * the 4,096-photon warm-up of a single GPU's larger passes) */
    GRM_OPT_WARMUP_SLACK = 12,
    /* 1 (default): a wave whose only work left is one photon hands it to the lone-photon kernel (two
     * waves per photon, after the launch); 0: the lane loop keeps it; 2: every photon is handed over
     * at the top of its first step (tests of the lone-photon path) */
    GRM_OPT_LONE = 13,
    /* photons of the first warm-up admission batch (default 64; later batches double the history) */
    GRM_OPT_WARMUP_BATCH = 14,
    /* a photon of this many steps (default 1500; 0 = off) leaves the lane loop at the top of a step
     * for a two-wave pair of the early worker, which runs beside the main transport launch on a
     * second stream */
    GRM_OPT_EARLY_STEPS = 15,
    /* test only: 1 launches the early worker on the transport stream ahead of the main launch, as a
     * kernel-serialising tool (a counter profiler) would run them; the worker must then leave */
    GRM_OPT_EARLY_SERIAL = 16,
    /* test only: != 0 makes the transport kernel's kernel-argument check fail (the failure path must
     * end the call with an error, no photon tracked) */
    GRM_OPT_KARG_TEST = 17,
    /* 18: retired (GRM_OPT_LONE_K, an experiment of round 3: no gain) */
    /* a wave claims at most this many photons of a warm-up admission batch at a time, spreading the
     * batch, and its photons' scattering families, over more waves (0: as many lanes as it has idle;
     * -1, the default: 4 in the 4,096-photon warm-up, 0 in the ramp of a small pass) */
    GRM_OPT_WARMUP_SPREAD = 19,
    /* 20, 21: retired (GRM_OPT_WARMUP_BLOCKS / _WAVES, round 4); setting them is an error */
    /* live bias: a transport call runs on at most (h + n) / this many lanes, n = the call's photons,
     * h = the photons tracked since the last reset (whole workgroups, at least one; default 96;
     * 0 = always the full grid).  bias_func's counters (harm_model.cpp:1391-1404) trail the claims by
     * the photons in flight, which matters only while the history behind them is short; measured at
     * 192^2, photon_n = 1e5 (1.45 M photons in one call, 96 seeds each): recorded +4.4 %
     * against the reference with 131 k lanes in flight, +2.3 % with 22.5 k (ratio 64), +1.0 % with
     * 16 k.  A bench pass (photon_n = 1e6, 14.5 M photons) keeps the full grid, and so do the later
     * batches of a pass fed in chunks; a frozen bias (GRM_OPT_BIAS_MODE = 1) always does.  A
     * multi-rank job's calls of fewer than 32 x the grid's lanes run at twice this ratio (their
     * concurrent ranks lag the job's history more). */
    GRM_OPT_FLIGHT_RATIO = 22,
    /* 23-27: the role-split bulk kernel's switches, in include/grmonty_amd_debug.h; only a variant build
     * (tools/build_variant.sh with -DGRM_WITH_SPLIT) accepts them */
    /* a multi-rank job (grm_engine_set_peers / grm_engine_link_peers): a pass's warm-up waits at most
     * this many ms for every rank's transport launch of the pass to start before its first claim, so
     * that no rank begins the job's warm-up alone (default 0 = no wait: ranks that run their passes
     * back to back stay uncoupled; the one-GPU emulation of N ranks, whose launches queue behind each
     * other, sets 500) */
    GRM_OPT_JOB_START_WAIT_MS = 28,
    /* 1 (default): the scattered child of a photon on a two-wave pair -- the early worker's
     * (GRM_OPT_EARLY_STEPS) or the lone kernel's (GRM_OPT_LONE) -- joins that kernel's queue of
     * children and starts on its next free pair at once, as the reference tracks a child as soon as
     * it is made (harm_model.cpp:1016-1023), instead of waiting for the overflow relaunch after the
     * kernel has ended; 0: every such child goes to the overflow relaunch */
    GRM_OPT_EARLY_CHILDREN = 29
};

/* --- engine lifecycle (super_photon.cuh:29-40) ------------------------------------------ */
/* fields: 8 row-major [n1][n2] arrays (x2 fastest): rho, u, u1, u2, u3, B1, B2, B3.
 * hotcross: (GRM_HC_N_W+1)*(GRM_HC_N_T+1) log10 sigma table; k2: GRM_N_E_SAMP+1 log K2 table.
 * scalars: bias_norm, x1_min (= log r_h), max_tau_scatt (initial), d_tau_k. */
int grm_engine_create(const grm_header *header, const double *const fields[8], const grm_units *units,
                      const double *hotcross, const double *k2, const double scalars[4], int device,
                      grm_engine **out);
void grm_engine_destroy(grm_engine *e);
const char *grm_engine_last_error(const grm_engine *e);
int grm_engine_set_option(grm_engine *e, int opt, int64_t value);

/* --- transport (super_photon.cuh:55-61) ------------------------------------------------- */
/* host batch -> device copy -> persistent transport; synchronous. */
int grm_engine_track(grm_engine *e, const grm_init_photon *batch, size_t n);
/* batch already resident in device memory (e.g. a torch tensor's data_ptr); synchronous. */
int grm_engine_track_device(grm_engine *e, const grm_init_photon *dev_batch, size_t n);
/* copy out accumulated spectrum [GRM_N_TH_BINS][GRM_N_E_BINS] and counters (does not reset). */
int grm_engine_finish(grm_engine *e, grm_spectrum_cell *spectrum_out, uint64_t *n_recorded, uint64_t *n_scatt,
                      double *max_tau_scatt);
/* zero the spectrum and counters; max_tau_scatt back to its initial value. */
int grm_engine_reset(grm_engine *e);
int grm_engine_stats(const grm_engine *e, grm_stats *out);
/* device pointer of the spectrum accumulator (GRM_N_TH_BINS*GRM_N_E_BINS cells), for in-place
 * collectives (RCCL all-reduce over xGMI) without a host round trip. */
void *grm_engine_spectrum_device_ptr(grm_engine *e);
/* copy the per-photon trace (requires GRM_OPT_TRACE_CAP > 0); returns records produced. */
int64_t grm_engine_trace(grm_engine *e, grm_trace *out, size_t cap);
/* copy a host batch into an engine-owned device buffer once (inputs resident in HBM); *dev_out is
 * valid for grm_engine_track_device until the next upload or destroy. */
int grm_engine_upload(grm_engine *e, const grm_init_photon *batch, size_t n, grm_init_photon **dev_out);

/* diagnostics (per-wave records, timing builds, watchdog records, raw counters) and the
 * per-function device probes of the parity tests: include/grmonty_amd_debug.h */

/* --- multi-GPU: one engine per GPU/process, RCCL over xGMI ------------------------------ */
/* rank 0 creates the 128-byte RCCL unique id and ships it to the others (any transport) */
int grm_rccl_unique_id(uint8_t id_out[128]);
int grm_engine_comm_init(grm_engine *e, const uint8_t id[128], int nranks, int rank);
/* in-place all-reduce of the spectrum (fp64 sum), counters (u64 sum) and max tau_scatt (max):
 * the only exchange step of the path (photon shards are independent). */
int grm_engine_allreduce(grm_engine *e);
/* One end-of-job exchange instead of one per pass: a rank runs its passes (run_simulation calls)
 * back to back, stashing each pass's results on the device (grm_engine_stash after the pass's
 * transport, into one of grm_engine_stash_reserve's slots), then ONE grouped RCCL all-reduce of all
 * slots (grm_engine_allreduce_stash: spectra and counters summed, max tau_scatt and longest life
 * maxed) and reads each pass's reduced result (grm_engine_stash_read).  The ranks' pass timelines
 * are then not coupled pass by pass (a rank with a long-lived photon in one pass does not hold the
 * others at that pass).  Same reduction as grm_engine_allreduce (harm_model.cpp:340-414 is one pass). */
int grm_engine_stash_reserve(grm_engine *e, int n_slots);
int grm_engine_stash(grm_engine *e, int slot);
/* slots [first, first + n_slots): a job reduces its warm-up slots and its timed slots separately,
 * each once (re-reducing a slot would multiply it by the rank count) */
int grm_engine_allreduce_stash(grm_engine *e, int first, int n_slots);
int grm_engine_stash_read(grm_engine *e, int slot, grm_spectrum_cell *spec, uint64_t *n_rec, uint64_t *n_scatt,
                          double *max_tau, uint64_t *n_steps);
/* The stash's raw words of slots [first, first + n_slots), in the engine's own packing, read
 * (write = 0) or written back (write = 1): per slot grm_stash_words(0) spectrum doubles (reduced by
 * sum), grm_stash_words(1) u64 words reduced by sum (recorded, scattered, steps, tracked, children,
 * overflow, dropped, primaries, lives > 1e5 steps) and grm_stash_words(2) reduced by max (max
 * tau_scatt bits, longest life).  A null array skips its part.  For a reduction over another
 * transport than RCCL (tests: gloo) with exactly grm_engine_allreduce_stash's semantics. */
int grm_engine_stash_raw(grm_engine *e, int first, int n_slots, double *spec, uint64_t *sums, uint64_t *maxs,
                         int write);
int grm_stash_words(int which);

/* The job's adaptive bias across ranks.  bias_func (harm_model.cpp:1391-1404) runs on the counters
 * of every photon recorded so far; a rank that saw only its own would run on a history N times
 * shorter (measured: +18 / +30 / +35 % recorded at 2 / 4 / 8 emulated ranks).  Each
 * engine keeps one counter block per pass slot (allocated by grm_engine_stash_reserve); with peers
 * set, the transport kernels read the SAME slot of every rank's blocks (remote ones over xGMI) and
 * run bias_func on their sums (max for max tau_scatt).
 *   grm_engine_begin_pass(e, slot): the next pass counts into block `slot` (reset first); slot < 0
 *     = the engine's private block, no sharing (the default).
 *   grm_engine_counters_ipc_handle: the 64-byte IPC handle of this engine's blocks, for the others;
 *   grm_engine_set_peers(e, handles[n][64], n, rank): open the other ranks' blocks (n <= 1: off);
 *   grm_engine_link_peers(engines, n): the same for n engines of one process on one device.
 *   grm_engine_job_counters(e, out[4]): bias_func's denominator, summed n_scatt, n_recorded and max
 *     tau_scatt of the current slot as the kernels see them (diagnostics / tests). */
int grm_engine_begin_pass(grm_engine *e, int slot);
int grm_engine_counters_ipc_handle(grm_engine *e, uint8_t out[64]);
int grm_engine_set_peers(grm_engine *e, const uint8_t *handles, int n, int rank);
int grm_engine_link_peers(grm_engine *const *engines, int n);
int grm_engine_job_counters(grm_engine *e, double out[4]);
/* 1 if device `device` can read device `peer`'s memory (hipDeviceCanAccessPeer; same device: 1) --
 * checked by bench.py for every rank's GPU before grm_engine_set_peers */
int grm_device_peer_ok(int device, int peer);

/* --- host model (harm_model.hpp; C++ host, no GPU) ------------------------------------- */
typedef struct grm_model grm_model;
/* HARMModel(photon_n, mass_unit) + read_file(path)   harm_model.cpp:64-232 */
int grm_model_load(const char *path, int photon_n, double mass_unit, grm_model **out);
void grm_model_free(grm_model *m);
const char *grm_model_last_error(void);
/* init(): geometry, hotcross, emission tables, weight, nint    harm_model.cpp:234-240 */
int grm_model_init(grm_model *m, int n_threads);
/* init() with the hotcross, K2 and nint / dndlnu_max tables built on GPU `device`
 * (csrc/grm_tables.hip; the reference's GPU builder is hotcross_table.cu:35-65); the rest as
 * grm_model_init.  grm_model_table_ms: GPU time of those builders (ms), 0 after grm_model_init. */
int grm_model_init_device(grm_model *m, int n_threads, int device);
double grm_model_table_ms(const grm_model *m);
void grm_model_header(const grm_model *m, grm_header *h);
void grm_model_units(const grm_model *m, grm_units *u);
/* bias_norm, x1_min, max_tau_scatt (initial), d_tau_k, rh */
void grm_model_scalars(const grm_model *m, double out[5]);
/* 0 rho 1 u 2 u1 3 u2 4 u3 5 B1 6 B2 7 B3 */
const double *grm_model_field(const grm_model *m, int which);
/* 0 hotcross 1 k2 2 f 3 weight 4 nint 5 dndlnu_max 6 det */
const double *grm_model_table(const grm_model *m, int which);
/* create an engine from a loaded + initialised model */
int grm_engine_create_from_model(const grm_model *m, int device, grm_engine **out);

/* Emission (harm_model.cpp:673-892): zone-parallel, deterministic for a given seed whatever
 * n_threads is (per-zone count draw, then one Philox stream per photon -- the same streams as
 * grm_engine_emit).  Returns photons written (<= cap) or -1 on error.
 * Call with out=NULL to only count (exact).  zone range [z0, z1) in row-major zone order
 * (z1 < 0 = all) -- used to shard emission across ranks. */
int64_t grm_model_emit(grm_model *m, uint64_t seed, int64_t z0, int64_t z1, grm_init_photon *out, size_t cap,
                       int n_threads);
/* the same for the zones z0, z0 + stride, z0 + 2 stride, ... < z1 (a strided shard: rank r of N
 * takes z0 = r, stride = N; the union over ranks is again exactly the single-GPU photon set) */
int64_t grm_model_emit_strided(grm_model *m, uint64_t seed, int64_t z0, int64_t z1, int64_t stride, grm_init_photon *out,
                               size_t cap, int n_threads);
/* cumulative expected photon count per zone, for balanced zone-range sharding (n1*n2 doubles) */
int grm_model_zone_weights(const grm_model *m, double *out);

/* --- device emission (harm_model.cpp:673-811, 1337-1389) -------------------------------- */
/* Per-zone emission record, built once per model on the host: init_zone's expected count and
 * dn_max, the zone centre (get_coord :1639-1644), get_fluid_zone's n_e / Theta_e / |B| and the
 * fluid-frame tetrad of sample_zone_photon (:717-731, tetrads.cpp:68-124).  272 B. */
typedef struct grm_emit_zone {
    double nz;             /* expected superphotons; 0 = the zone emits nothing */
    double dn_max;
    double x[4];
    double n_e, theta_e, b;
    double e_con[4][4];    /* tetrad basis vectors e_(b)^mu, row b */
    double e_cov_t[4];     /* e_cov[b][0], b = 0..3 (photon energy, :773) */
    double e_cov_z[4];     /* e_cov[b][3], b = 0..3 (angular momentum, :775) */
    double pad_;
} grm_emit_zone;

/* zone records [z0, z1) (z1 < 0 = all zones) into out[z1 - z0] */
int grm_model_zone_table(const grm_model *m, int64_t z0, int64_t z1, grm_emit_zone *out, int n_threads);
/* upload the zone table (all n1*n2 zones) and the weight / F emission tables (GRM_N_E_SAMP+1 each,
 * log values as in grm_model_table 3 and 2) to the engine */
int grm_engine_emit_setup(grm_engine *e, const grm_emit_zone *zones, int64_t n_zones, const double *weight,
                          const double *f);
int grm_engine_emit_setup_from_model(grm_engine *e, const grm_model *m);
/* Emit every superphoton of zones [z0, z1) on the GPU (make_super_photon / sample_zone_photon):
 * zone counts by stochastic rounding of nz with the zone stream's first draw, then one lane per
 * photon on its own Philox stream (key = seed, counter = (draw, photon-in-zone + 1, zone, 'EMIT')).
 * The same photons as grm_model_emit (up to device libm rounding).  *dev_out = engine-owned device
 * buffer valid until the next emit or destroy; synchronous. */
int grm_engine_emit(grm_engine *e, uint64_t seed, int64_t z0, int64_t z1, grm_init_photon **dev_out,
                    uint64_t *n_out);
/* the zones z0, z0 + stride, ... < z1 (grm_model_emit_strided's set, the same photons) */
int grm_engine_emit_strided(grm_engine *e, uint64_t seed, int64_t z0, int64_t z1, int64_t stride,
                            grm_init_photon **dev_out, uint64_t *n_out);
/* device -> host copy of n photons from an engine buffer (tests, writers) */
int grm_engine_download(grm_engine *e, const grm_init_photon *dev, size_t n, grm_init_photon *host_out);

/* report_spectrum (harm_model.cpp:416-471): 200 rows x 37 columns "%10.5g ".
 * out2 (optional): luminosity, max tau_scatt. */
int grm_write_spectrum(const grm_model *m, const grm_spectrum_cell *spectrum, const char *path, double out2[2]);
/* statistics sidecar of the spectrum file (not in the reference): 200 rows of
 * log10(E) then, per theta bin, nph (recorded superphotons), dn_dle (sum w) and de_dle (sum w E),
 * "%.17g" -- what an effective-N / KS comparison of two spectra needs and the 37-column file lacks. */
int grm_write_spectrum_stats(const grm_model *m, const grm_spectrum_cell *spectrum, const char *path);

/* ABI introspection: sizes of the POD structs (0 header 1 units 2 init_photon 3 spectrum_cell
 * 4 trace 5 stats 6 emit_zone) */
size_t grm_sizeof(int which);
const char *grm_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GRMONTY_AMD_H */
