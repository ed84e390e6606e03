/*
 * grmonty_oracle.h -- C-ABI of the CPU ORACLE (test infrastructure only).
 *
 * This library is a plain-C++ restatement of the reference's CPU transport
 * path (m-torhan/cuda-grmonty, cuda_grmonty/harm_model.cpp and friends).  It
 * exists to CHECK the HIP product path; it is never linked, loaded or called
 * by the product.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - tetrads / proba / monty_rand / integration: pinned bit-exact against the
 *     reference's own sources compiled here (oracle/_ref, recipe oracle/Makefile).
 *   - harm_model / radiation / hotcross / jnu_mixed: the reference files need
 *     spdlog + std::format (absent from this image) and are unbuildable here;
 *     these restatements are pinned by independent mathematics (scipy Bessel
 *     K2, finite-difference Christoffel symbols, metric inverse identity,
 *     Klein-Nishina limits) and by the reference's own dump-parser fixture.
 *
 * All structs are POD and mirror the reference layouts (harm_data.hpp,
 * photon.hpp) so the same bytes can be handed to the product C-ABI.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* harm_data.hpp:19-44 (Header) */
typedef struct grmo_header {
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
} grmo_header;

/* harm_data.hpp:62-71 (Units) */
typedef struct grmo_units {
    double mass_unit, l_unit, t_unit, rho_unit, u_unit, b_unit, theta_e_unit, n_e_unit;
} grmo_units;

/* photon.hpp:41-52 (InitPhoton) -- 15 doubles + int, padded to 128 B */
typedef struct grmo_init_photon {
    double x[4];
    double k[4];
    double w, e, l, n_e_0, theta_e_0, b_0, e_0;
    int n_scatt;
    int pad_;
} grmo_init_photon;

/* harm_data.hpp:129-143 (Spectrum) -- 13 doubles, reference field order */
typedef struct grmo_spectrum {
    double dn_dle, de_dle, nph, nscatt, x1i_av, x2i_sq, x3f_sq, tau_abs, tau_scatt, ne_0, theta_e_0, b_0, e_0;
} grmo_spectrum;

/* harm_data.hpp:117-125 (FluidParams) */
typedef struct grmo_fluid {
    double n_e, theta_e, b;
    double u_con[4], u_cov[4], b_con[4], b_cov[4];
} grmo_fluid;

/* per-photon end-of-life record, used to compare trajectories photon-by-photon */
typedef struct grmo_trace {
    uint64_t id;
    uint64_t parent_id;
    double w, e, x1, x2, x3, tau_abs, tau_scatt;
    int32_t n_scatt;
    int32_t n_step;
    int32_t end_reason; /* 0 recorded, 1 escaped-not-binned, 2 horizon/absorbed/roulette, 3 max-step, 4 invalid */
    int32_t ix2;
    int32_t i_e;
    int32_t pad_;
} grmo_trace;

enum { GRMO_RNG_MT19937 = 0, GRMO_RNG_PHILOX = 1 };
enum { GRMO_BIAS_LIVE = 0, GRMO_BIAS_FROZEN = 1 };

typedef struct grmo_model grmo_model;

/* ---- model (harm_model.cpp:64-232) ---- */
grmo_model *grmo_model_new(int photon_n, double mass_unit);
void grmo_model_free(grmo_model *m);
int grmo_model_read_file(grmo_model *m, const char *path); /* 0 ok */
/* direct construction from arrays (used for component tests) */
int grmo_model_set(grmo_model *m, const grmo_header *h, const double *const fields[8]);
void grmo_model_get_header(const grmo_model *m, grmo_header *h);
void grmo_model_get_units(const grmo_model *m, grmo_units *u);
/* scalars: bias_norm, rh, x1_min, max_tau_scatt, d_tau_k */
void grmo_model_get_scalars(const grmo_model *m, double out[5]);
void grmo_model_set_max_tau_scatt(grmo_model *m, double v);
const double *grmo_model_field(const grmo_model *m, int which); /* 0..7: rho,u,u1,u2,u3,b1,b2,b3 */

/* ---- init tables (harm_model.cpp:234-338, hotcross.cpp:60-79, jnu_mixed.cpp:57-73) ---- */
void grmo_init_geometry(grmo_model *m);
void grmo_init_hotcross(grmo_model *m, int n_threads); /* threads only split rows; per-entry math is serial */
void grmo_init_emiss_tables(grmo_model *m);
void grmo_init_weight_table(grmo_model *m);
void grmo_init_nint_table(grmo_model *m);
void grmo_init_all(grmo_model *m, int n_threads);
const double *grmo_table(const grmo_model *m, int which); /* 0 hotcross(221*81) 1 k2 2 f 3 weight 4 nint 5 dndlnu_max 6 det */
void grmo_set_table(grmo_model *m, int which, const double *src); /* load a table computed elsewhere */

/* ---- component functions (for parity tests) ---- */
void grmo_gcov(const grmo_model *m, const double x[4], double g[16]);
void grmo_gcon(const grmo_model *m, const double x[4], double g[16]);
void grmo_connection(const grmo_model *m, const double x[4], double lconn[64]);
void grmo_init_dkdlam(const grmo_model *m, const double x[4], const double k[4], double dk[4]);
double grmo_step_size(const grmo_model *m, const double x[4], const double k[4]);
/* state[13] = x[4], k[4], dkdlam[4], e_0_s ; in/out */
void grmo_push_photon(const grmo_model *m, double state[13], double dl);
void grmo_fluid_params(const grmo_model *m, const double x[4], grmo_fluid *out);
double grmo_bk_angle(const double k[4], const grmo_fluid *f, double b_unit);
double grmo_fluid_nu(const double k[4], const double u_cov[4]);
double grmo_alpha_inv_scatt(const grmo_model *m, double nu, double theta_e, double n_e);
double grmo_alpha_inv_abs(const grmo_model *m, double nu, double theta_e, double n_e, double b, double theta);
double grmo_hotcross_lookup(const grmo_model *m, double w, double theta_e);
double grmo_hotcross_num(double w, double theta_e);
double grmo_synch(const grmo_model *m, double nu, double n_e, double theta_e, double b, double theta);
double grmo_k2_eval(const grmo_model *m, double theta_e);
double grmo_f_eval(const grmo_model *m, double theta_e, double b, double nu);
void grmo_make_tetrad(const double u_con[4], const double trial[4], const double g_cov[16], double e_con[16],
                      double e_cov[16]);
void grmo_boost(const double v[4], const double u[4], double vp[4]);
double grmo_gk61(int which_fn, double param, double a, double b, double eps_abs, double eps_rel, int max_iv);

/* ---- RNG-driven samplers (rng_mode: MT19937 seeded `seed`, or Philox stream (seed, id)) ---- */
typedef struct grmo_rng grmo_rng;
grmo_rng *grmo_rng_new(int mode, uint64_t seed, uint64_t id);
void grmo_rng_free(grmo_rng *r);
double grmo_rng_uniform(grmo_rng *r);
double grmo_rng_chi_sq(grmo_rng *r, int dof);
uint64_t grmo_rng_counter(const grmo_rng *r);
void grmo_sample_electron(grmo_rng *r, const double k[4], double p[4], double theta_e);
double grmo_sample_klein_nishina(grmo_rng *r, double k0);
double grmo_sample_thomson(grmo_rng *r);
void grmo_sample_rand_dir(grmo_rng *r, double out[3]);
void grmo_sample_scattered(grmo_rng *r, const double k[4], const double p_in[4], double kp[4]);
/* philox4x32-10 block (for known-answer tests) */
void grmo_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint64_t grmo_child_id(uint64_t parent_id, uint64_t parent_ctr);

/* ---- transport ---- */
/* Track a batch of emitted photons (harm_model.cpp:366-404 body + track_super_photon).
 * rng_mode PHILOX: photon i uses stream id = id_base + i, children derive ids (grmo_child_id).
 * rng_mode MT19937: a single mt19937(seed) stream shared in call order (reference semantics).
 * bias_mode FROZEN: bias_func uses (scatt0, rec0, max_tau0) for the whole batch (device-parity mode).
 * trace may be NULL; otherwise up to trace_cap end-of-life records are written.
 * Returns number of trace records produced (may exceed trace_cap; excess dropped). */
int64_t grmo_track_batch(grmo_model *m, const grmo_init_photon *ph, size_t n, int rng_mode, uint64_t seed,
                         uint64_t id_base, int bias_mode, uint64_t scatt0, uint64_t rec0, double max_tau0,
                         grmo_trace *trace, size_t trace_cap);
/* Concurrency emulator: the batch tracked as a concurrent engine schedules it -- `slots` photons
 * advanced round-robin one loop iteration (harm_model.cpp:919-1063) per round, bias_func reading
 * counter snapshots taken every `refresh` rounds, children either tracked depth-first in their
 * parent's slot (the reference recursion, :1023) or deferred to a LIFO stack shared by `group`
 * slots (the device's wave stacks), primaries claimed in the device's interleaved order
 * (claim_sh: 2^sh runs; -1 = the engine's rule) under its warm-up admission (warm_n photons in
 * batches b0, b0, 2 b0, ... each opened when in flight <= admitted >> slack; warm_n -1 = slots)
 * and an optional cap on photons in flight.  Philox streams (id = id_base + index).  One slot,
 * depth-first, refresh 1 is the serial reference operation for operation.  timeline (6 doubles
 * per row: round, claims, recorded, scattered, max tau_scatt, in flight) every `timeline` rounds.
 * Returns the number of rounds. */
enum {
    GRMO_EMU_SLOTS = 0,
    GRMO_EMU_GROUP = 1,
    GRMO_EMU_REFRESH = 2,
    GRMO_EMU_CHILD_MIN = 3,
    GRMO_EMU_DEPTH_FIRST = 4,
    GRMO_EMU_CLAIM_SH = 5,
    GRMO_EMU_WARM_N = 6,
    GRMO_EMU_WARM_SLACK = 7,
    GRMO_EMU_WARM_B0 = 8,
    GRMO_EMU_FLIGHT_CAP = 9,
    GRMO_EMU_TIMELINE = 10,
    GRMO_EMU_NCFG = 11
};
int64_t grmo_track_concurrent(grmo_model *m, const grmo_init_photon *batch, size_t n, uint64_t seed,
                              uint64_t id_base, const int64_t *cfg, size_t n_cfg, grmo_trace *trace,
                              size_t trace_cap, double *timeline, size_t timeline_cap, int64_t *n_timeline);
int64_t grmo_last_trace_count(const grmo_model *m); /* trace records the last traced call produced */
void grmo_reset_spectrum(grmo_model *m);
void grmo_set_spectrum(grmo_model *m, const grmo_spectrum in[6 * 200]);
void grmo_get_spectrum(const grmo_model *m, grmo_spectrum out[6 * 200]);
/* counters: created, scattered, recorded ; plus steps (transport loop iterations) */
void grmo_get_counters(const grmo_model *m, uint64_t out[4]);

/* ---- emission (harm_model.cpp:673-811, 1337-1389) ---- */
/* Emit up to cap photons with the reference's serial zone walk and mt19937(seed).
 * Returns the number emitted; *done = 1 when the zone walk is exhausted. */
int64_t grmo_emit(grmo_model *m, uint64_t seed, grmo_init_photon *out, size_t cap, int *done);
void grmo_init_zone(const grmo_model *m, int i, int j, double out[2]); /* nz, dn_max */
/* Emission with the product's per-photon Philox streams (photon-by-photon check of grm_model_emit
 * and grm_engine_emit): zones [z0, z1) (z1 < 0 = all), count draw = slot 0 of the zone stream,
 * photon p = slot p + 1.  out = NULL counts only; returns the number of photons. */
int64_t grmo_emit_philox(grmo_model *m, uint64_t seed, int64_t z0, int64_t z1, grmo_init_photon *out, size_t cap);

/* ---- whole run, reference CPU semantics (main.cpp:43-53, harm_model.cpp:340-414) ---- */
/* run_simulation with mt19937(123) shared by emission and transport, live counters. */
double grmo_run_simulation(grmo_model *m, uint64_t seed); /* returns wall seconds */
double grmo_run_simulation_traced(grmo_model *m, uint64_t seed, grmo_trace *trace, size_t trace_cap,
                                  int64_t *n_trace);
int grmo_report_spectrum(const grmo_model *m, const char *path, double out_lum_maxtau[2]);

size_t grmo_sizeof(int which); /* 0 header 1 units 2 init_photon 3 spectrum 4 fluid 5 trace */

#ifdef __cplusplus
}
#endif
