/*
 * grm_split.hip -- the bulk transport kernel with the roles split between waves (split_kernel).
 *
 * track_kernel (grm_engine.hip) runs track_super_photon's loop (harm_model.cpp:919-1063) as a lane
 * state machine: every lane owns a photon and makes one push attempt per trip, and the lanes whose
 * attempt completed a step then run the interaction block (fluid gather, absorption / scattering
 * coefficients, bias, decision, :937-1056) together.  Only ~68 % of attempts complete a step (the rest
 * are push_photon's halving sub-steps, :1279-1285), so that block -- about half of a trip's
 * instructions -- issues with ~41 of 64 lanes, and each wave's trip is one long dependent chain of
 * fp64 work and two L2 round trips that the second wave of its SIMD covers only in part (VALU-active
 * 0.34 of wave cycles).
 *
 * Here a workgroup of 512 lanes is four PAIRS of waves, the two waves of pair g on the same SIMD
 * (waves g and g + 4).  Lane l of pair g owns photon p = 64 g + l in both of them:
 *   - the GEOMETRY wave (g) runs the photon's geodesic -- photon_2, step_size, push_photon with its
 *     halving (:920-930, :1217-1289, :1620-1630) -- one push attempt per lane per loop trip, no
 *     global memory at all, and publishes every completed step into a per-photon ring of SP_R slots
 *     in LDS (the state after the push, the step size, and the point's trig values, from which the
 *     metric there is two dozen flops);
 *   - the INTERACTION wave (g + 4) consumes the ring in order -- stop criteria with their roulette
 *     draws (:919, :932), the fluid and the radiation coefficients at the step's end point, bias_func,
 *     the scattering decision and the weight (:937-1063) -- once most of its lanes have a step ready,
 *     so that block issues with (nearly) every lane active; it also owns everything else of a
 *     photon's life: refills (primaries, scattered children from the wave's stack), records, counters,
 *     the warm-up admission, the hand-overs to the lone and early kernels.
 * The geodesic does not depend on the interactions except at a scattering: the interaction wave then
 * asks the geometry lane to re-push photon_2 (the ring slot before the step) by dl * frac to the
 * scattering point (:1005-1010), which is published as the head of a new generation of slots, and the
 * photon continues from there (steps pushed ahead on the old geodesic are discarded by their tag).  A
 * new photon is a request too: its start state goes into the slot before the generation's head and
 * the geometry lane publishes the set-up (dk/dlambda from a zero-length attempt, :915, :1571-1587).
 *
 * Ring protocol (per photon, all in LDS, [slot][field][photon] so a wave's accesses are consecutive
 * 8-B words): slot q % SP_R holds step q of the lane's sequence, tagged (generation << 32 | q), data
 * written before the tag (a wave's LDS operations complete in order).  cons = the next slot the
 * interaction lane consumes; slot cons - 1 is photon_2 of step cons and stays live, so the geometry
 * lane writes slot q only when q <= cons + SP_R - 2.  A request (generation, kind, q0) restarts the
 * geometry lane from slot q0 - 1: kind NEW (set-up), SCATTER (re-push by s_len), IDLE (stop).
 *
 * RNG draws, their order and every arithmetic operation of a photon are those of transport_trip, so a
 * frozen-bias batch equals the oracle photon by photon as the lane loop does
 * (tests/test_gpu_transport.py[split]).
 */
#define GRM_SPLIT_TU 1
/* only the interaction waves record: four record buffers per workgroup, indexed by the wave's pair */
#include <hip/hip_runtime.h>
__shared__ int s_recidx[8]; /* wave -> its pair (interaction waves) */
#define GRM_REC_WAVES 4
#define GRM_REC_WAVE(t) (s_recidx[(t) >> 6])
#include "grm_engine.hip"

namespace {

constexpr int SP_PAIRS = 4;
constexpr int SP_BLOCK = 128 * SP_PAIRS; /* threads: SP_PAIRS geometry waves, then SP_PAIRS interaction waves */
constexpr int SP_PH = 64 * SP_PAIRS;     /* photons per workgroup */
#ifndef GRM_SPLIT_RING
#define GRM_SPLIT_RING 4
#endif
constexpr int SP_R = GRM_SPLIT_RING; /* ring slots per photon: the geometry runs up to SP_R - 2 steps ahead */
enum : int {
    SF_X1, SF_X2, SF_X3, SF_K0, SF_K1, SF_K2, SF_K3, SF_DK0, SF_DK1, SF_DK2, SF_DK3, SF_E0S, SF_DL,
    SF_R1, SF_C2X, SF_STH, SF_CTH, SP_F
};
constexpr unsigned SK_NEW = 0, SK_SCATTER = 1, SK_IDLE = 2;
constexpr int E_SETUP = 0, E_SP = 1, E_STEP = 2; /* what an interaction lane expects in its next slot */
constexpr int GS_IDLE = 0, GS_START = 1, GS_PUSH = 2;

__shared__ double s_ring[SP_R * SP_F * SP_PH];
__shared__ unsigned long long s_tag[SP_R * SP_PH];
__shared__ unsigned long long s_req[SP_PH]; /* (generation << 32) | (kind << 30) | q0 */
__shared__ double s_len[SP_PH];             /* SCATTER: the re-push length dl * frac */
__shared__ unsigned s_cons[SP_PH];
__shared__ int s_exit[SP_PAIRS];
__shared__ int s_swtop[SP_PAIRS];
__shared__ int s_simd[SP_BLOCK / 64];

/* diagnostic build (-DGRM_TIMING): wave-level accounting into Ctl.timing, slots 0-7 interaction waves
 * (loop trips, evaluation rounds, ready lanes in them, active lanes in them, cycles in the evaluation,
 * cycles in all, waiting trips, trips that refilled), 8-15 geometry waves (loop trips, trips with a
 * push, pushing lanes, lanes held by a full ring, idle lanes, cycles in all, cycles in the push,
 * idle trips) */
#ifdef GRM_TIMING
#define SP_T(v, x) (v) += (x)
#else
#define SP_T(v, x) do { } while (0)
#endif

__device__ __forceinline__ double &ring(int slot, int f, int p) { return s_ring[(slot * SP_F + f) * SP_PH + p]; }
__device__ __forceinline__ int slot_of(uint32_t q) { return (int)(q % (uint32_t)SP_R); }

/* the state (x^1..3, k, dk/dlambda, e_0_s) of slot s */
__device__ __forceinline__ void ring_load_state(int s, int p, double x[4], double k[4], double dk[4], double &e0s) {
    x[0] = 0.0; /* x^0 enters no result (see make_sreq) */
    x[1] = ring(s, SF_X1, p);
    x[2] = ring(s, SF_X2, p);
    x[3] = ring(s, SF_X3, p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        k[i] = ring(s, SF_K0 + i, p);
        dk[i] = ring(s, SF_DK0 + i, p);
    }
    e0s = ring(s, SF_E0S, p);
}

/* ------------------------------------------------------------------------------------------- */
/* geometry wave                                                                                 */
/* ------------------------------------------------------------------------------------------- */
__device__ void sp_geometry(KArgsK *ka, int pair, int p, unsigned long long &trips) {
    double x[4] = {0.0, 0.0, 0.0, 0.0}, k[4] = {0.0, 0.0, 0.0, 0.0}, dk[4] = {0.0, 0.0, 0.0, 0.0}, e0s = 0.0;
    double bx[4], bkk[4], bdk[4]; /* the attempt's start at depth > 0 (:1222-1228); depth 0 restarts from the ring */
    unsigned long long cur = 0;   /* the request in force */
    uint32_t gen = 0, q = 0;      /* q: the slot the next completed push goes to */
    int st = GS_IDLE;
    bool setup = false, head = false; /* head: the push in progress is a generation's head (set-up or scattering point) */
    double dl = 0.0;
    int depth = 0;
    uint32_t pend = 0;
    unsigned idle_spins = 0;
#ifdef GRM_TIMING
    unsigned long long tg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long tg0 = __builtin_amdgcn_s_memtime();
#endif
    while (true) {
        KArgsK *const kt = karg_fresh(ka);
        const Params &P = karg_params(kt);
        ++trips;
        SP_T(tg[0], 1);
        if (__hip_atomic_load(&s_exit[pair], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        const unsigned long long r = __hip_atomic_load(&s_req[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (r != cur) {
            cur = r;
            gen = (uint32_t)(r >> 32);
            q = (uint32_t)r & 0x3fffffffu;
            const unsigned kind = (unsigned)(r >> 30) & 3u;
            if (kind == SK_IDLE) {
                st = GS_IDLE;
            } else {
                ring_load_state(slot_of(q + SP_R - 1), p, x, k, dk, e0s); /* photon_2 / the start state */
                setup = kind == SK_NEW;
                head = true;
                dl = setup ? 0.0 : s_len[p];
                depth = 0;
                pend = 0;
                st = GS_PUSH;
            }
        }
        if (st == GS_START) {
            /* photon_2 of the step is slot q - 1 (the last one written); slot q must be free */
            const uint32_t cons = __hip_atomic_load(&s_cons[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            SP_T(tg[3], (unsigned long long)__popcll(__ballot((int)(q - cons) > SP_R - 2)));
            if ((int)(q - cons) <= SP_R - 2) {
                dl = step_size(P, x, k); /* :927, 1620-1630 */
                depth = 0;
                pend = 0;
                setup = false;
                st = GS_PUSH;
            }
        }
        const bool push = st == GS_PUSH;
        SP_T(tg[4], (unsigned long long)__popcll(__ballot(st == GS_IDLE)));
        {
            /* push once most live lanes can (an attempt issues the same instructions for 1 lane as for
             * 64, and they are issue slots the interaction wave on this SIMD does not get), or after a
             * few sleeps */
            const int n_push = __popcll(__ballot(push));
            const int n_live = __popcll(__ballot(st != GS_IDLE));
            const Ctl &C = karg_ctl(kt);
            if (n_push == 0 || (n_push < ((n_live * C.split_gthr) >> 6) && idle_spins < (unsigned)C.split_spin)) {
                SP_T(tg[7], 1);
                if (n_push || idle_spins < 4)
                    __builtin_amdgcn_s_sleep(1);
                else
                    __builtin_amdgcn_s_sleep(4);
                ++idle_spins;
                continue;
            }
        }
        idle_spins = 0;
        SP_T(tg[1], 1);
        SP_T(tg[2], (unsigned long long)__popcll(__ballot(push)));
#ifdef GRM_TIMING
        const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
#endif
        if (push) {
            /* one attempt of push_photon at the current node of its halving tree (:1217-1289); the
             * set-up's attempt has zero length: x, k stay, dk = dk/dlambda at x (init_dkdlam) */
            Trig T;
            bool have_t = false, again = false;
            if (setup || !(x[1] < P.xs1)) {
                if (depth > 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        bx[i] = x[i];
                        bkk[i] = k[i];
                        bdk[i] = dk[i];
                    }
                }
                double e_1;
                Gcov G;
                const bool fail = push_attempt(P, x, k, dk, e0s, ldexp(dl, -depth), e_1, T, G);
                const int s0 = slot_of(q + SP_R - 1);
                if (setup) {
                    /* restore x, k exactly (a non-finite dk must not leak into them through 0 * dk) */
                    x[1] = ring(s0, SF_X1, p);
                    x[2] = ring(s0, SF_X2, p);
                    x[3] = ring(s0, SF_X3, p);
#pragma unroll
                    for (int i = 0; i < 4; ++i) k[i] = ring(s0, SF_K0 + i, p);
                } else if (fail && depth < MAX_SUBDIV) {
                    if (depth == 0) {
                        double e_r;
                        ring_load_state(s0, p, x, k, dk, e_r);
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            x[i] = bx[i];
                            k[i] = bkk[i];
                            dk[i] = bdk[i];
                        }
                    }
                    ++depth;
                    pend |= 1u << depth;
                    again = true;
                }
                if (!again) {
                    if (!setup) e0s = e_1;
                    have_t = true;
                }
            }
            if (!again && pend) { /* the pending second half of the deepest level */
                depth = 31 - __builtin_clz(pend);
                pend &= ~(1u << depth);
                again = true;
            }
            if (!again) {
                if (!have_t) trig_at(P, x, T);
                /* publish, unless a request arrived during the attempt (a result published just before
                 * a request carries the old generation's tag, which the interaction lane skips) */
                if (__hip_atomic_load(&s_req[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == cur) {
                    const int s1 = slot_of(q);
                    ring(s1, SF_X1, p) = x[1];
                    ring(s1, SF_X2, p) = x[2];
                    ring(s1, SF_X3, p) = x[3];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        ring(s1, SF_K0 + i, p) = k[i];
                        ring(s1, SF_DK0 + i, p) = dk[i];
                    }
                    ring(s1, SF_E0S, p) = e0s;
                    ring(s1, SF_DL, p) = dl;
                    ring(s1, SF_R1, p) = T.r1;
                    ring(s1, SF_C2X, p) = T.c2x;
                    ring(s1, SF_STH, p) = T.sth;
                    ring(s1, SF_CTH, p) = T.cth;
                    __asm__ volatile("" ::: "memory"); /* the data before the tag (LDS completes in order) */
                    __hip_atomic_store(&s_tag[s1 * SP_PH + p], ((unsigned long long)gen << 32) | q,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                ++q;
                /* a step ending outside [x1_min, x1_max] (or at NaN) ends the photon at its stop test
                 * after the push (:932).  A head has no such test: the loop-top test (:919) of the step
                 * after it ends the photon, so that step is pushed (and discarded) all the same */
                st = (!head && (x[1] < P.x1_min || x[1] > P.x1_max || isnan(x[1]))) ? GS_IDLE : GS_START;
                head = false;
            }
        }
#ifdef GRM_TIMING
        tg[6] += __builtin_amdgcn_s_memtime() - tp0;
#endif
    }
#ifdef GRM_TIMING
    tg[5] = __builtin_amdgcn_s_memtime() - tg0;
    if ((threadIdx.x & 63) == 0) {
        const Ctl &C = karg_ctl(karg_fresh(ka));
        for (int i = 0; i < 8; ++i) atomicAdd(C.timing + 8 + i, tg[i]);
    }
#endif
}

/* ------------------------------------------------------------------------------------------- */
/* interaction wave                                                                              */
/* ------------------------------------------------------------------------------------------- */
/* post a request to the photon's geometry lane */
__device__ __forceinline__ void sp_request(int p, uint32_t gen, unsigned kind, uint32_t q0) {
    __asm__ volatile("" ::: "memory");
    __hip_atomic_store(&s_req[p],
                       ((unsigned long long)gen << 32) | ((unsigned long long)kind << 30) | (unsigned long long)q0,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void sp_export(LoneRec *r, int s, int p, double w, double tau_abs, double tau_scatt,
                                          double a_si, double a_ai, double bi, double fl_ne, const Cold *cold,
                                          const Rng &rng, int n_step, int n_scatt) {
    double2 *d = reinterpret_cast<double2 *>(r);
    d[0] = make_double2(0.0, ring(s, SF_X1, p));
    d[1] = make_double2(ring(s, SF_X2, p), ring(s, SF_X3, p));
    d[2] = make_double2(ring(s, SF_K0, p), ring(s, SF_K1, p));
    d[3] = make_double2(ring(s, SF_K2, p), ring(s, SF_K3, p));
    d[4] = make_double2(ring(s, SF_DK0, p), ring(s, SF_DK1, p));
    d[5] = make_double2(ring(s, SF_DK2, p), ring(s, SF_DK3, p));
    d[6] = make_double2(w, ring(s, SF_E0S, p));
    d[7] = make_double2(tau_abs, tau_scatt);
    d[8] = make_double2(a_si, a_ai);
    d[9] = make_double2(bi, fl_ne);
    const double2 *c = reinterpret_cast<const double2 *>(cold);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) d[10 + qq] = c[qq];
    r->id = rng.id;
    r->ctr = rng.ctr;
    r->n_step = n_step;
    r->n_scatt = n_scatt;
    r->pad = 0;
}

__device__ void sp_interaction(KArgsK *ka, const Params &P0, const Ctl &C0, int pair, int p, bool karg_bad,
                               unsigned long long &wave_trips, unsigned long long &wave_steps, unsigned &o_tracked,
                               unsigned &o_primaries, unsigned &o_children, unsigned &o_nstep_max, unsigned &o_long) {
    const unsigned lane_id = threadIdx.x & 63;
    const uint64_t gtid = (uint64_t)blockIdx.x * SP_BLOCK + threadIdx.x;
    SReq *wstack = C0.stack + (gtid >> 6) * WSTACK_CAP; /* the wave's own (allocated for every wave) */
    int *wtop = &s_swtop[pair];
    Cold *cold = C0.cold + gtid;
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
    /* the photon */
    bool active = false;
    int expect = E_STEP;
    uint32_t gen = 0, cons = 1; /* slot 0 = the first photon's start state */
    double w = 0.0, tau_abs = 0.0, tau_scatt = 0.0, a_si = 0.0, a_ai = 0.0, bi = 0.0, fl_ne = 0.0, x1_cur = 0.0;
    double p_dtau_abs = 0.0, p_dtau_scatt = 0.0, p_wc = 0.0;
    int n_step = 0, n_scatt = 0, flight = 0;
    Rng rng;
    rng.k0 = C0.key0;
    rng.k1 = C0.key1;
    rng.id = 0;
    rng.ctr = rng.ctr_hi = 0;
    unsigned c_tracked = 0, c_primaries = 0, c_children = 0, c_nstep_max = 0, c_long = 0;
    bool pool_done = karg_bad;
    unsigned long long res_next = 0, res_end = 0;
    bool head_done = false;
    bool warm = !karg_bad && C0.admit_n != 0;
    unsigned wait_trips = 0, spins = 0;
    int n_round = 0; /* ready lanes of the round's first slot */
    double bias_d = bias_den(P0, C0);
    unsigned trip = 1;
    const unsigned long long lt_mask = (lane_id == 0) ? 0ull : (~0ull >> (64 - lane_id));
    __hip_atomic_store(&s_cons[p], cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef GRM_TIMING
    unsigned long long ti[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tj[4] = {0, 0, 0, 0}; /* evaluation: to the fluid, fluid, radiation, the rest */
    unsigned long long tk[3] = {0, 0, 0};    /* loop top + refill, hand-overs, readiness (all trips) */
    const unsigned long long ti0 = __builtin_amdgcn_s_memtime();
#endif

    while (true) {
        KArgsK *const kt = karg_fresh(ka);
        const Params &P = karg_params(kt);
        const Ctl &C = karg_ctl(kt);
        ++wave_trips;
        SP_T(ti[0], 1);
#ifdef GRM_TIMING
        const unsigned long long tl0 = __builtin_amdgcn_s_memtime();
#endif
        if (warm && blockIdx.x >= WARM_BLOCKS) { /* the warm-up's batches go to the first workgroups */
            unsigned long long end = 0;
            if (lane_id == 0) end = __hip_atomic_load(C.admit_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane((int)(end >> 32)) != -1 ||
                __builtin_amdgcn_readfirstlane((int)end) != -1) {
                __builtin_amdgcn_s_sleep(127);
                continue;
            }
            warm = false;
            if (!C.bias_frozen) bias_d = bias_den(P, C);
        }
        if ((trip++ & (REFRESH_TRIPS - 1)) == 0 || warm) {
            flush_counters(C);
            if (!C.bias_frozen) bias_d = bias_den(P, C);
            if (C.watchdog_ticks) {
                bool stop = __hip_atomic_load(&C.ctr->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (!stop && __builtin_amdgcn_s_memrealtime() - rt_start > C.watchdog_ticks) {
                    stop = true;
                    if (lane_id == 0) __hip_atomic_store(&C.ctr->abort, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (stop) {
                    if (lane_id == 0) __hip_atomic_store(C.admit_end, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (lane_id == 0 && C.n_peers > 1) atomicOr(C.in_flight, WARM_DONE);
                    if (active) {
                        const unsigned long long slot = atomicAdd(C.stuck_count, 1ull);
                        if (slot < C.stuck_cap) {
                            const int s = slot_of(cons + SP_R - 1);
                            double *r = C.stuck + slot * STUCK_WORDS;
                            r[0] = (double)rng.id;
                            r[1] = n_step;
                            r[2] = expect;
                            r[3] = r[4] = 0.0;
                            r[5] = w;
                            r[6] = ring(s, SF_E0S, p);
                            r[7] = ring(s, SF_DL, p);
                            r[8] = 0.0;
                            r[9] = ring(s, SF_X1, p);
                            r[10] = ring(s, SF_X2, p);
                            r[11] = ring(s, SF_X3, p);
                            for (int i = 0; i < 4; ++i) r[12 + i] = ring(s, SF_K0 + i, p);
                        }
                        atomicAdd(&C.ctr->n_abandoned, 1ull);
                        active = false;
                    }
                    pool_done = true;
                    warm = false;
                    if (lane_id == 0) *wtop = 0;
                }
            }
        }
        if (__builtin_amdgcn_readfirstlane(s_recn[pair]) >= RECBUF_FLUSH) flush_records(C);
        /* Refill (converged point): the claim logic of track_kernel (primaries as soon as refill_min
         * lanes are idle, children from the wave's stack in batches of child_min, the warm-up's
         * admission batches); a photon's set-up is a NEW request to its geometry lane */
        const unsigned long long idle = __ballot(!active);
        if (idle) {
            int top = *wtop;
            if (top > WSTACK_CAP) top = WSTACK_CAP;
            const int n_idle = __popcll(idle);
            const bool none_active = idle == __ballot(1);
            const bool child_due = top >= C.child_min || (pool_done && top > 0);
            int k_child = 0, k_pool = 0;
            bool go;
            if (none_active || child_due) {
                k_child = n_idle < top ? n_idle : top;
                k_pool = pool_done ? 0 : n_idle - k_child;
                go = none_active || n_idle >= min(C.child_min, top);
            } else {
                k_pool = pool_done ? 0 : n_idle;
                go = k_pool >= C.refill_min;
            }
            if (go) {
                const int r = __popcll(idle & lt_mask);
                unsigned long long base = 0;
                if (k_pool > 0) {
                    if (warm) {
                        long long got = 0;
                        int off = 0;
                        const bool job = C.n_peers > 1;
                        unsigned long long j_hist = 0;
                        long long j_flight = 0;
                        if (job) warm_job(C, j_hist, j_flight);
                        const unsigned long long unit = job ? WARM_HIST + 1 : 1;
                        if (lane_id == 0) {
                            const unsigned long long end =
                                __hip_atomic_load(C.admit_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (end == ~0ull) {
                                off = 1;
                            } else {
                                const unsigned long long head =
                                    __hip_atomic_load(C.pool_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                base = head;
                                if (head < end) {
                                    unsigned long long want = min((unsigned long long)k_pool, end - head);
                                    if (C.admit_spread) want = min(want, C.admit_spread);
                                    atomicAdd(C.in_flight, want * unit);
                                    if (atomicCAS(C.pool_head, head, head + want) == head)
                                        got = (long long)want;
                                    else
                                        atomicAdd(C.in_flight, (unsigned long long)(-(long long)(want * unit)));
                                } else if (job ? (unsigned long long)j_flight <= (j_hist >> C.admit_slack)
                                               : __hip_atomic_load(C.in_flight, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <=
                                                     ((C.admit_h0 + end) >> C.admit_slack)) {
                                    const unsigned long long h = job ? j_hist : C.admit_h0 + end;
                                    const unsigned long long grow =
                                        job ? min(h, C.admit_lim - min(h, C.admit_lim)) / (unsigned long long)C.n_peers
                                            : min(h, C.admit_lim - h);
                                    const unsigned long long next =
                                        (end >= C.admit_n || (job && h >= C.admit_lim))
                                            ? ~0ull
                                            : min(C.admit_n, end + max(C.admit_b0, grow));
                                    const bool opened = atomicCAS(C.admit_end, end, next) == end;
                                    if (opened && next == ~0ull && job) atomicOr(C.in_flight, WARM_DONE);
                                    if (opened && C.phases) {
                                        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                                        if (next == ~0ull) C.phases[0] = t;
                                        const unsigned long long kk = atomicAdd(C.phases + 2, 1ull);
                                        if (kk < (PHASE_LOG - 3) / 2) {
                                            C.phases[3 + 2 * kk] = t;
                                            const unsigned long long f =
                                                __hip_atomic_load(C.in_flight, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                            const long long fl = job ? (long long)(int)(unsigned)f : (long long)f;
                                            C.phases[4 + 2 * kk] = (unsigned long long)(fl < 0 ? 0 : fl);
                                        }
                                    }
                                }
                            }
                        }
                        if (__shfl(off, 0)) {
                            warm = false;
                        } else {
                            base = __shfl(base, 0);
                            k_pool = (int)__shfl(got, 0);
                            if (k_pool > 0 && base + k_pool >= C.pos_end) pool_done = true;
                        }
                    }
                    if (!warm) {
                        if (res_next >= res_end) {
                            unsigned long long b = 0;
                            if (lane_id == 0) b = atomicAdd(C.pool_head, (unsigned long long)RES_CHUNK);
                            b = __shfl(b, 0);
                            res_next = b;
                            res_end = min(b + RES_CHUNK, C.pos_end);
                            head_done = b + RES_CHUNK >= C.pos_end;
                            if (C.phases && lane_id == 0 && b < C.pos_end && head_done)
                                C.phases[1] = __builtin_amdgcn_s_memrealtime();
                        }
                        base = res_next;
                        k_pool = res_end > res_next ? (int)min((unsigned long long)k_pool, res_end - res_next) : 0;
                        res_next += k_pool;
                        if (head_done && res_next >= res_end) pool_done = true;
                    }
                }
                if (lane_id == 0) *wtop = top - k_child;
                SP_T(ti[7], (k_child + k_pool) > 0 ? 1 : 0);
                bool has = false, ok = true;
                double x[4], k[4];
                if (!active && r < k_child) {
                    SReq R;
                    load_sreq(wstack + (top - 1 - r), R);
                    ok = sample_child_core(P, R, rng, x, k, w, cold);
                    n_scatt = R.n_scatt;
                    if (!ok && C.trace)
                        write_trace(C, cold, R.id, R.w, R.x[1], R.x[2], R.x[3], 0.0, 0.0, R.n_scatt, 0, 4, -1, -1);
                    has = true;
                }
                if (!active && r >= k_child && r - k_child < k_pool) {
                    const unsigned long long pos = base + (unsigned long long)(r - k_child);
                    const unsigned long long idx = (pos & ((1ull << C.pool_sh) - 1)) * C.pool_m + (pos >> C.pool_sh);
                    if (pos < C.pos_end && idx >= C.n_pool) --flight; /* a hole: claimed, ends at once */
                    if (pos < C.pos_end && idx < C.n_pool) {
                        if (C.pool_kind == 0) {
                            load_primary_core(C, idx, rng, x, k, w, cold);
                            n_scatt = 0;
                            ++c_primaries;
                        } else {
                            SReq R;
                            load_sreq(reinterpret_cast<const SReq *>(C.pool) + idx, R);
                            ok = sample_child_core(P, R, rng, x, k, w, cold);
                            n_scatt = R.n_scatt;
                            if (!ok && C.trace)
                                write_trace(C, cold, R.id, R.w, R.x[1], R.x[2], R.x[3], 0.0, 0.0, R.n_scatt, 0, 4,
                                            -1, -1);
                        }
                        has = true;
                    }
                }
                if (has) {
                    ++c_tracked;
                    n_step = 0;
                    tau_abs = tau_scatt = 0.0;
                    if (ok) {
                        /* photon set-up (harm_model.cpp:895-917): the validity check here, dk/dlambda from the
                         * geometry lane's zero-length attempt, the coefficients at the head slot below */
                        if (isnan(x[0]) || isnan(x[1]) || isnan(x[2]) || isnan(x[3]) || isnan(k[0]) || isnan(k[1]) ||
                            isnan(k[2]) || isnan(k[3]) || w == 0.0) {
                            if (C.trace) write_trace(C, cold, rng.id, w, x[1], x[2], x[3], 0.0, 0.0, n_scatt, 0, 4, -1, -1);
                        } else {
                            const int s = slot_of(cons + SP_R - 1);
                            ring(s, SF_X1, p) = x[1];
                            ring(s, SF_X2, p) = x[2];
                            ring(s, SF_X3, p) = x[3];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                ring(s, SF_K0 + i, p) = k[i];
                                ring(s, SF_DK0 + i, p) = 0.0;
                            }
                            ring(s, SF_E0S, p) = cold->e;
                            ++gen;
                            sp_request(p, gen, SK_NEW, cons);
                            expect = E_SETUP;
                            active = true;
                        }
                    }
                    if (!active) --flight; /* started and ended at once (invalid) */
                }
            }
        }
#ifdef GRM_TIMING
        const unsigned long long tl1 = __builtin_amdgcn_s_memtime();
        tk[0] += tl1 - tl0; /* loop top: refresh, record flush, refill */
#endif
        if (!__any(active)) {
            if (warm) {
                int d = flight;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
                if (lane_id == 0 && d) atomicAdd(C.in_flight, (unsigned long long)(long long)d);
                flight = 0;
            }
            if (pool_done && *wtop == 0) break;
            if (warm) {
                if (++wait_trips > (1u << 21) && lane_id == 0) {
                    __hip_atomic_store(C.admit_end, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (C.n_peers > 1) atomicOr(C.in_flight, WARM_DONE);
                }
                __builtin_amdgcn_s_sleep(16);
            }
            continue;
        }
        wait_trips = 0;
        /* hand-overs at the top of a step (the photon's state = slot cons - 1): a photon of early_steps
         * steps to the concurrent early_kernel; a wave's last photon to lone_kernel */
        if (C.early_q && !warm) {
            const bool early = active && expect == E_STEP && n_step >= C.early_steps;
            if (__ballot(early) && __hip_atomic_load(C.early_live, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT) == 1 &&
                __hip_atomic_load(C.early_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < C.early_cap && early) {
                const unsigned long long slot = atomicAdd(C.early_tail, 1ull);
                if (slot < C.early_cap) {
                    sp_export(C.early_q + slot, slot_of(cons + SP_R - 1), p, w, tau_abs, tau_scatt, a_si, a_ai, bi,
                              fl_ne, cold, rng, n_step, n_scatt);
                    __threadfence();
                    __hip_atomic_store(C.early_ready + slot, C.early_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    active = false;
                    ++gen;
                    sp_request(p, gen, SK_IDLE, cons);
                }
            }
        }
        const bool tail = pool_done && !warm;
        if ((tail || C.lone_all) && C.lone) {
            const unsigned long long act = __ballot(active);
            const bool alone = __popcll(act) == 1 && *wtop == 0;
            if (alone || C.lone_all) {
                const bool hand = active && expect == E_STEP &&
                                  __hip_atomic_load(C.lone_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < C.lone_cap;
                if (__ballot(hand)) {
                    unsigned long long slot = ~0ull;
                    if (hand) slot = atomicAdd(C.lone_count, 1ull);
                    const bool handed = hand && slot < C.lone_cap;
                    if (handed) {
                        sp_export(C.lone + slot, slot_of(cons + SP_R - 1), p, w, tau_abs, tau_scatt, a_si, a_ai, bi,
                                  fl_ne, cold, rng, n_step, n_scatt);
                        active = false;
                        ++gen;
                        sp_request(p, gen, SK_IDLE, cons);
                    }
                    if (__ballot(handed)) continue;
                }
            }
        }
#ifdef GRM_TIMING
        const unsigned long long tl2 = __builtin_amdgcn_s_memtime();
        tk[1] += tl2 - tl1; /* hand-overs */
#endif
        /* the steps ready: wait until most active lanes have one (the block then issues with nearly
         * every lane), or a few sleeps */
        /* a round evaluates up to split_batch consecutive slots per lane: after the first, the lanes
         * whose next slot is ready too go on at once (no loop top, refill or readiness wait between)
         * while at least half the lanes of the round do */
        bool spin_again = false;
        for (int bj = 0; bj < C.split_batch; ++bj) {
        const int sc = slot_of(cons);
        const bool ready =
            active && (bj == 0 || expect == E_STEP) &&
            __hip_atomic_load(&s_tag[sc * SP_PH + p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) ==
                (((unsigned long long)gen << 32) | cons);
        if (bj > 0) {
            if (__popcll(__ballot(ready)) * 2 < n_round) break;
        } else {
            const int n_ready = __popcll(__ballot(ready));
            const int n_act = __popcll(__ballot(active));
            const int need = max(1, (n_act * C.split_thr) >> 6);
#ifdef GRM_TIMING
            tk[2] += __builtin_amdgcn_s_memtime() - tl2; /* readiness */
#endif
            if (n_ready == 0 || (n_ready < need && spins < (unsigned)C.split_spin)) {
                ++spins;
                SP_T(ti[6], 1);
                __builtin_amdgcn_s_sleep(1);
                spin_again = true;
                break; /* to the loop top (the batch loop's continue would not get there) */
            }
            spins = 0;
            n_round = n_ready;
            SP_T(ti[1], 1);
            SP_T(ti[2], (unsigned long long)n_ready);
            SP_T(ti[3], (unsigned long long)n_act);
        }
#ifdef GRM_TIMING
        const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
#endif
        bool stepped = false;
        if (ready) {
            const double x1 = ring(sc, SF_X1, p);
            bool ended = false, scattered = false;
            int end_at = -1;  /* end of life by a stop test: 0 = at the current state (:919), 1 = at the step's end (:932) */
            int reason = -1;  /* else the trace reason */
            if (expect == E_STEP) {
                stepped = true;
                if (stop_criterion(P, x1_cur, w, rng)) { /* :919 */
                    ended = true;
                    end_at = 0;
                    stepped = false;
                } else if (stop_criterion(P, x1, w, rng)) { /* :932-934 */
                    ended = true;
                    end_at = 1;
                } else if (isnan(x1)) { /* NaN position: absorbing, ended at once (see transport_trip) */
                    atomicAdd(&C.ctr->n_nan, 1ull);
                    ended = true;
                    reason = 3;
                }
            }
            if (!ended && (expect != E_STEP || a_ai > 0.0 || a_si > 0.0 || fl_ne > 0.0)) {
                /* the fluid and the absorption / scattering coefficients at the slot's point: the step's
                 * end (:938-975), the scattering point (:1012-1039) or the set-up point (:904-913) */
                const double xv[4] = {0.0, x1, ring(sc, SF_X2, p), ring(sc, SF_X3, p)};
                double kv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) kv[i] = ring(sc, SF_K0 + i, p);
                Trig T;
                T.r1 = ring(sc, SF_R1, p);
                T.s2x = 0.0; /* not used by the metric */
                T.c2x = ring(sc, SF_C2X, p);
                T.sth = ring(sc, SF_STH, p);
                T.cth = ring(sc, SF_CTH, p);
                Gcov G;
                gcov_from_trig(P, T, G);
#ifdef GRM_TIMING
                const unsigned long long tq0 = __builtin_amdgcn_s_memtime();
#endif
                ZoneFetch Z;
                zone_fetch(P, xv, Z);
                Fluid F;
                fluid_from(P, xv, G, Z, F);
                fl_ne = F.n_e;
#ifdef GRM_TIMING
                const unsigned long long tq1 = __builtin_amdgcn_s_memtime();
                if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) {
                    tj[0] += tq0 - tp0;
                    tj[1] += tq1 - tq0;
                }
#endif
                const bool at_sp = expect == E_SP, setup = expect == E_SETUP;
                if (at_sp && F.n_e > 0.0 && (kv[0] > 1.0e5 || kv[0] < 0.0 || isnan(kv[0]) || isnan(kv[1]) || isnan(kv[3]))) {
                    w = 0.0; /* scatter_super_photon's parent-side check (:1076-1081) */
                    ended = true;
                    reason = 2;
                } else {
                    const double nu = fluid_nu(kv, F);
                    const bool zero = !setup && (nu < 0.0 || (!at_sp && F.n_e == 0.0));
                    double a_s = 0.0, a_a = 0.0;
                    if (!zero) radiation_coeffs(P, kv, F, nu, a_s, a_a);
                    const double bf = (zero && !at_sp) ? 0.0 : bias_func(bias_d, F.theta_e, w);
#ifdef GRM_TIMING
                    if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1)
                        tj[2] += __builtin_amdgcn_s_memtime() - tq1;
#endif
                    if (setup) {
                        a_si = a_s;
                        a_ai = a_a;
                        bi = bf;
                    } else if (at_sp) {
                        /* the child leaves as a scatter request (:1015-1024) */
                        if (F.n_e > 0.0) {
                            if (push_request(C, xv, kv, rng, n_scatt, cold, F, p_wc, wstack, wtop)) ++flight;
                            ++c_children;
                        }
                        a_si = a_s;
                        a_ai = a_a;
                        bi = bf;
                        tau_abs += p_dtau_abs;
                        tau_scatt += p_dtau_scatt;
                    } else {
                        /* trapezoid optical depths over the step (:957-975) */
                        const double dl = ring(sc, SF_DL, p);
                        double d_tau_scatt, d_tau_abs, bias;
                        if (zero) {
                            d_tau_scatt = 0.5 * a_si * P.d_tau_k * dl;
                            d_tau_abs = 0.5 * a_ai * P.d_tau_k * dl;
                            bias = 0.0;
                        } else {
                            d_tau_scatt = 0.5 * (a_si + a_s) * P.d_tau_k * dl;
                            d_tau_abs = 0.5 * (a_ai + a_a) * P.d_tau_k * dl;
                            bias = 0.5 * (bi + bf);
                        }
                        a_si = a_s;
                        a_ai = a_a;
                        bi = bf;
                        /* x1 = -log u (:983), settled without the logarithm when possible */
                        const double u = uniform(rng);
                        const double bdt = bias * d_tau_scatt;
                        const bool may = bdt > (1.0 - u) * (1.0 - 0x1p-40);
                        const double lx = may ? -flog(u) : 0.0;
                        const double wc = fdiv(w, bias);
                        if (may && bdt > lx && wc > WEIGHT_MIN) { /* :985 */
                            const double frac = fdiv(lx, bias * d_tau_scatt);
                            d_tau_abs *= frac;
                            if (d_tau_abs > 100) { /* absorbed before scattering */
                                ended = true;
                                reason = 2;
                            } else {
                                d_tau_scatt *= frac;
                                const double d_tau = d_tau_abs + d_tau_scatt;
                                if (d_tau_abs < 1.0e-3)
                                    w *= (1.0 - d_tau * (1.0 / 24.0) * (24.0 - d_tau * (12.0 - d_tau * (4.0 - d_tau))));
                                else
                                    w *= fexp(-d_tau);
                                /* photon_2 re-pushed by dl * frac to the scattering point (:1005-1010): by
                                 * the geometry lane, from slot cons - 1, as the head of a new generation */
                                s_len[p] = dl * frac;
                                ++gen;
                                sp_request(p, gen, SK_SCATTER, cons);
                                p_dtau_abs = d_tau_abs;
                                p_dtau_scatt = d_tau_scatt;
                                p_wc = wc;
                                expect = E_SP;
                                scattered = true;
                            }
                        } else if (d_tau_abs > 100) { /* absorbed */
                            ended = true;
                            reason = 2;
                        } else {
                            const double d_tau = d_tau_abs + d_tau_scatt;
                            if (d_tau < 1.0e-3)
                                w *= (1.0 - d_tau * (1.0 / 24.0) * (24.0 - d_tau * (12.0 - d_tau * (4.0 - d_tau))));
                            else
                                w *= fexp(-d_tau);
                            tau_abs += d_tau_abs;
                            tau_scatt += d_tau_scatt;
                        }
                    }
                }
            }
            if (!ended && !scattered) {
                if (expect == E_SETUP) {
                    expect = E_STEP;
                } else {
                    ++n_step; /* :1058-1063 */
                    if (n_step > MAX_N_STEP) {
                        ended = true;
                        reason = 3;
                    }
                    expect = E_STEP;
                }
                if (!ended) {
                    x1_cur = x1;
                    ++cons;
                }
            }
            if (ended) {
                /* the end of the photon's life: recorded (record_criterion :1066, record_super_photon)
                 * or traced with its reason, at the state the reference ends it in */
                const int se = end_at == 0 ? slot_of(cons + SP_R - 1) : sc;
                const double ex1 = end_at == 0 ? x1_cur : x1, ex2 = ring(se, SF_X2, p), ex3 = ring(se, SF_X3, p);
                if (end_at >= 0 && ex1 > P.x1_max && n_step <= MAX_N_STEP)
                    record_photon(P, C, cold, rng.id, w, ex1, ex2, ex3, tau_abs, tau_scatt, n_scatt, n_step, spec_slice(C),
                                  SPEC_CELL);
                else if (C.trace)
                    write_trace(C, cold, rng.id, w, ex1, ex2, ex3, tau_abs, tau_scatt, n_scatt, n_step,
                                reason < 0 ? 2 : reason, -1, -1);
                active = false;
                --flight;
                c_nstep_max = max(c_nstep_max, (unsigned)n_step);
                c_long += n_step > 100000 ? 1u : 0u;
                ++gen;
                sp_request(p, gen, SK_IDLE, cons);
            }
        }
        __hip_atomic_store(&s_cons[p], cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef GRM_TIMING
        ti[4] += __builtin_amdgcn_s_memtime() - tp0;
#endif
        wave_steps += (unsigned long long)__popcll(__ballot(stepped));
        }
        if (spin_again) continue;
        if (warm) {
            int d = flight;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
            if (lane_id == 0 && d) atomicAdd(C.in_flight, (unsigned long long)(long long)d);
            flight = 0;
        }
    }
#ifdef GRM_TIMING
    ti[5] = __builtin_amdgcn_s_memtime() - ti0;
    if (lane_id == 0)
        for (int i = 0; i < 8; ++i) atomicAdd(C0.timing + i, ti[i]);
    /* the per-phase sums were kept by varying first lanes: reduce them over the wave */
    for (int i = 0; i < 3; ++i) {
        unsigned long long v = tj[i];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane_id == 0) atomicAdd(C0.timing + 44 + i, v);
    }
    if (lane_id == 0)
        for (int i = 0; i < 3; ++i) atomicAdd(C0.timing + 32 + i, tk[i]);
#endif
    o_tracked = c_tracked;
    o_primaries = c_primaries;
    o_children = c_children;
    o_nstep_max = c_nstep_max;
    o_long = c_long;
}

__global__ __launch_bounds__(SP_BLOCK, 1) void split_kernel(Params P_, Ctl C_) {
    KArgsK *const ka = kargs();
    const Ctl &C0 = C_;
    const Params &P0 = P_;
    const int wave = threadIdx.x >> 6;
    const unsigned lane_id = threadIdx.x & 63;
    /* Roles.  split 1: waves 0-3 geometry, 4-7 interaction (pair g = waves g, g + 4: the same SIMD when
     * the waves are dealt round-robin).  split 2: by the SIMD each wave runs on (HW_ID), the geometry
     * waves on SIMDs 0-1 and the interaction waves on SIMDs 2-3, two of a kind per SIMD (one wave's
     * latency covered by the other's work of the same kind); pair g = the g-th wave of each role;
     * a placement other than two waves per SIMD falls back to split 1. */
    int pair = wave & (SP_PAIRS - 1);
    bool geo = wave < SP_PAIRS;
    if (C0.split_mode == 2) {
        unsigned simd;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 4, 2)" : "=s"(simd));
        if (lane_id == 0) s_simd[wave] = (int)simd;
        __syncthreads();
        int n_geo = 0, rank = 0, per[4] = {0, 0, 0, 0};
        const bool g = simd < 2;
        for (int v = 0; v < SP_BLOCK / 64; ++v) {
            const int sv = s_simd[v] & 3;
            ++per[sv];
            n_geo += sv < 2 ? 1 : 0;
            if (v < wave && (sv < 2) == g) ++rank;
        }
        if (n_geo == SP_PAIRS && per[0] == 2 && per[1] == 2 && per[2] == 2 && per[3] == 2) {
            geo = g;
            pair = rank;
        }
    }
    const int p = pair * 64 + (int)lane_id;
    const uint64_t gtid = (uint64_t)blockIdx.x * SP_BLOCK + threadIdx.x;
    if (lane_id == 0) s_recidx[wave] = pair;
    __syncthreads();
    /* ring tags and requests start empty (generation 0 is never requested: the first is 1) */
    for (int i = threadIdx.x; i < SP_R * SP_PH; i += SP_BLOCK) s_tag[i] = ~0ull;
    if (threadIdx.x < SP_PH) {
        s_req[threadIdx.x] = 0;
        s_cons[threadIdx.x] = 1;
    }
    if (threadIdx.x < SP_PAIRS) {
        s_exit[threadIdx.x] = 0;
        s_swtop[threadIdx.x] = 0;
        s_recn[threadIdx.x] = 0;
    }
    if (threadIdx.x < 4 * SP_PAIRS) s_cnt[threadIdx.x >> 2][threadIdx.x & 3] = 0;
    if (threadIdx.x == 0 && C0.early_q) __hip_atomic_store(C0.bulk_live, 1ull, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
    /* a failed argument check ends the interaction wave at once (the geometry wave follows it) */
    const bool karg_bad = !kargs_check(ka, P0, C0);
    unsigned long long trips = 0, steps = 0;
    unsigned c_tracked = 0, c_primaries = 0, c_children = 0, c_nstep_max = 0, c_long = 0;
    if (geo) {
        sp_geometry(ka, pair, p, trips);
    } else {
        if (karg_bad && lane_id == 0) atomicAdd(&C0.ctr->karg_bad, 1ull);
        sp_interaction(ka, P0, C0, pair, p, karg_bad, trips, steps, c_tracked, c_primaries, c_children, c_nstep_max,
                       c_long);
        if (lane_id == 0) __hip_atomic_store(&s_exit[pair], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        flush_counters(C0);
        flush_records(C0);
    }
    const Ctl &C = C0;
    __syncthreads();
    double *slice = spec_slice(C);
    for (int i = threadIdx.x; i < SPEC_LDS; i += SP_BLOCK) {
        if ((i & (SPEC_CELL - 1)) >= SPEC_FIELDS) continue;
        const double v = __hip_atomic_load(slice + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v != 0.0) slice[i] = 0.0;
        if (v != 0.0) unsafeAtomicAdd(reinterpret_cast<double *>(C.spec + i / SPEC_CELL) + (i & (SPEC_CELL - 1)), v);
    }
    unsigned long long w_tracked = c_tracked, w_primaries = c_primaries, w_children = c_children, w_long = c_long,
                       w_nstep_max = c_nstep_max;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        w_tracked += __shfl_xor(w_tracked, off);
        w_primaries += __shfl_xor(w_primaries, off);
        w_children += __shfl_xor(w_children, off);
        w_long += __shfl_xor(w_long, off);
        w_nstep_max = max(w_nstep_max, (unsigned long long)__shfl_xor(w_nstep_max, off));
    }
    if (lane_id == 0) {
        if (!geo) {
            atomicAdd(&C.ctr->n_steps, steps);
            atomicAdd(&C.ctr->n_tracked, w_tracked);
            atomicAdd(&C.ctr->n_primaries, w_primaries);
            atomicAdd(&C.ctr->n_children, w_children);
            if (w_long) atomicAdd(&C.ctr->n_long, w_long);
            atomicMax(&C.ctr->max_nstep, w_nstep_max);
        }
        if (C.waves) {
            unsigned long long *wr = C.waves + (gtid >> 6) * 4;
            wr[0] = rt_start;
            wr[1] = __builtin_amdgcn_s_memrealtime();
            wr[2] = trips;
            wr[3] = w_tracked;
        }
    }
    if (C.early_q) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(C.wg_exit, 1ull) == gridDim.x - 1)
                __hip_atomic_store(C.early_done, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

} /* namespace */

extern "C" hipError_t grm_split_launch(unsigned grid, hipStream_t s, const void *P, size_t p_size, const void *C,
                                       size_t c_size) {
    if (p_size != sizeof(grm::Params) || c_size != sizeof(Ctl)) return hipErrorInvalidValue; /* built apart */
    grm::Params p;
    Ctl c;
    memcpy(&p, P, sizeof p);
    memcpy(&c, C, sizeof c);
    hipLaunchKernelGGL(split_kernel, dim3(grid), dim3(SP_BLOCK), 0, s, p, c);
    return hipGetLastError();
}
