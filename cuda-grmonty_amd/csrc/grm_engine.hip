/*
 * grm_engine.hip -- persistent-wavefront superphoton transport for MI355X (gfx950)
 * and the C-ABI engine entry points (include/grmonty_amd.h).
 *
 * Replaces the reference's 2-stream x 16384-slot lock-step pipeline of nine kernels
 * per geodesic step with host refills and host re-queueing of scattered photons
 * (super_photon.cu:505-1037).  Here ONE kernel launch tracks a whole batch:
 *
 *   - each lane owns one superphoton in VGPRs for its whole life
 *     (track_super_photon, harm_model.cpp:894-1069, CPU semantics);
 *   - idle lanes refill first from their own child stack, then from the batch pool
 *     with one wave-aggregated atomic per refill (ballot + popcount);
 *   - a scattering pushes the child onto the lane's private stack in HBM (no
 *     inter-lane synchronisation); a full stack spills to an overflow pool that
 *     the host relaunches over (double-buffered) until empty;
 *   - escaping photons are binned with fp64 global atomics (record_super_photon,
 *     harm_model.cpp:1291-1335); counters are u64 (fixes SURVEY Q7).
 *
 * RNG: Philox4x32-10 stream per photon id (key = seed); a child's stream id is a
 * function of its parent's id and draw counter, so results do not depend on lane
 * assignment or scheduling (bias mode FROZEN makes a batch fully reproducible).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include <rccl/rccl.h>

#include "grm_device.h"
#include "grm_emit.h"

using namespace grm;

namespace {

/* One workgroup per CU of 512 lanes: two waves per SIMD at 256 VGPRs each -- the second wave issues
 * while the first waits on a gather or a scalar/branch slot (+20% over one wave per SIMD, measured
 * on MI355X).  The per-lane state copies and per-step lane fields take the LDS, so the
 * spectrum goes to a per-workgroup slice in HBM (L2 atomics). */
#define GRM_BLOCK 512
constexpr int BLOCK = GRM_BLOCK;
constexpr int MIN_WAVES_PER_SIMD = BLOCK / 256;
constexpr int STACK_DEPTH = 16;                 /* scatter-request slots per lane ... */
constexpr int WSTACK_CAP = 64 * STACK_DEPTH;    /* ... pooled into one stack per wave (192 KB of HBM) */

/* 192-B scatter request (three aligned 64-B segments per request): the state at a scattering event from which the child
 * photon is sampled later (scatter_super_photon, harm_model.cpp:1071-1145).
 * Lane stacks and overflow pools hold these. */
struct alignas(16) SReq {
    double x[4], k[4];          /* parent position / wave vector at the scattering point */
    double u_con[4], b_con[4];  /* fluid 4-velocity and b^mu there */
    double b, theta_e;          /* |B| (Gauss), Theta_e there */
    double w;                   /* child weight w_parent / bias */
    double n_e_0, theta_e_0;
    uint64_t id, parent;        /* child stream id, parent stream id */
    int32_t n_scatt, pad0;
};
static_assert(sizeof(SReq) == 192, "SReq layout");

/* 64-B per-lane cold photon fields (touched only at birth, scattering and recording): one aligned
 * segment per write.  The Photon fields l and e_0 (photon.hpp:19-36) are carried by the reference
 * but enter no result -- record_super_photon never accumulates e_0 and nothing reads l
 * (harm_model.cpp:1291-1335) -- so the lanes do not carry them. */
struct alignas(16) Cold {
    double e, x1i, x2i, n_e_0, theta_e_0, b_0;
    uint64_t parent;
    double pad;
};
static_assert(sizeof(Cold) == 64, "Cold layout");

struct DevCounters {
    unsigned long long n_recorded, n_scatt, max_tau_bits, n_steps;
    unsigned long long n_tracked, n_children, n_overflow, n_dropped;
    unsigned long long n_primaries, max_nstep, n_long, n_abandoned, abort, n_nan;
    unsigned long long karg_bad; /* track_kernel's kernel-argument check failed (see kargs_check) */
    /* a multi-rank job's warm-up state of this rank for the others' admission gates (pass blocks
     * only, see warm_job): photons admitted << 32 + photons in flight (signed), WARM_DONE once the
     * rank's admission is over */
    unsigned long long warm;
};
static_assert(sizeof(DevCounters) == 16 * 8, "DevCounters layout (grm_engine_debug_counters)");
constexpr unsigned long long WARM_DONE = 1ull << 63, WARM_HIST = 1ull << 32;
/* set by the rank's transport launch as it starts (the job's start barrier, job_started) */
constexpr unsigned long long WARM_STARTED = 1ull << 62;


struct LoneRec;
struct Ctl {
    const void *pool;      /* grm_init_photon[] (kind 0) or SReq[] (kind 1) */
    int pool_kind;
    unsigned long long n_pool;
    unsigned long long *pool_head;
    /* claim order: the head counts claim positions; position q < pos_end holds pool photon
     * (q mod 2^pool_sh) * pool_m + q / 2^pool_sh (a hole when that is >= n_pool).  Primaries are
     * interleaved over 2^pool_sh evenly spaced runs of the zone-ordered batch (see run_transport) */
    unsigned long long pos_end, pool_m;
    int pool_sh;
    uint64_t id_base;
    uint32_t key0, key1;
    SReq *stack;           /* [lanes][STACK_DEPTH] */
    Cold *cold;            /* [lanes] */
    SReq *ovf;             /* overflow out */
    unsigned long long ovf_cap;
    unsigned long long *ovf_count;
    grm_spectrum_cell *spec;
    double *spec_blocks;   /* [grid][SPEC_LDS] per-workgroup spectrum slices (when not in LDS), kept zero */
    DevCounters *ctr;
    grm_trace *trace;
    unsigned long long trace_cap;
    unsigned long long *trace_count;
    int bias_frozen;
    double f_scatt, f_rec, f_maxtau;
    unsigned long long *timing; /* GRM_TIMING builds: per-region wave cycles */
    int refill_min;             /* idle lanes a wave gathers before it takes primaries */
    int child_min;              /* children a wave gathers (on its stack and idle lanes) per sampling batch */
    /* Live-bias warm-up inside the launch: the first admit_n pool photons go in batches, each
     * admitted only when everything started before it (children included) has ended, and as large
     * as the history behind it (64, 64, 128, 256, ...): bias_func's running counters then evolve as
     * in the serial reference (harm_model.cpp:1391-1404).  *admit_end = end of the admitted batch
     * (~0 = no limit), *in_flight = photons started and not ended (children counted when pushed). */
    unsigned long long admit_n, admit_h0, admit_lim;
    int admit_slack;
    unsigned long long admit_b0; /* first batch */
    unsigned long long admit_spread; /* photons one wave claims at most per warm-up claim (0: no cap) */
    unsigned long long *admit_end, *in_flight;
    unsigned long long *waves;  /* per-wave record of the launch: start, exit (s_memrealtime), trips, photons */
    unsigned long long *phases; /* s_memrealtime when the warm-up admission ended ([0]) and the pool's
                                 * last claim chunk was taken ([1]); null = not recorded */
    int lanes;
    /* watchdog: a launch older than watchdog_ticks (s_memrealtime, 100 MHz; 0 = off) abandons its
     * photons and exits, so no input can keep the GPU busy without bound.  The first stuck_cap
     * abandoned lanes leave a STUCK_WORDS-double record (grm_engine_debug_stuck). */
    unsigned long long watchdog_ticks;
    double *stuck;
    unsigned long long stuck_cap, *stuck_count;
    /* lone photons handed over to lone_kernel (null = never); lone_all: every photon is handed over
     * at the top of its first step (GRM_OPT_LONE = 2: tests of the lone path) */
    LoneRec *lone;
    unsigned long long lone_cap, *lone_count;
    int lone_all;
    /* early hand-over of long photons to the concurrent early_kernel (early_q null = off): a photon
     * of >= early_steps steps at the top of a step; slots claimed by *early_tail, published by
     * early_ready[slot] = early_tag; *wg_exit counts exited workgroups, the last sets *early_done;
     * *early_live: 1 once early_kernel runs (no hand-over before, so none can strand), 2 when it
     * closed the queue because the bulk launch had not started (kernels serialised, e.g. under a
     * counter profiler); *bulk_live: set by every bulk workgroup as it starts */
    LoneRec *early_q;
    unsigned long long *early_ready, early_cap, early_tag;
    unsigned long long *early_tail, *early_head, *early_done, *wg_exit, *early_live, *bulk_live;
    int early_steps;
    /* a multi-rank pass's warm-up waits at most this long (s_memrealtime ticks, 100 MHz) for every
     * peer's launch of the pass to start before its first claim (0: no wait; GRM_OPT_JOB_START_WAIT_MS) */
    unsigned long long start_wait_ticks;
    int karg_test; /* test only (GRM_OPT_KARG_TEST): the kernel-argument check expects lanes + this */
    /* The job's bias counters across ranks: peers[r] = rank r's array of per-pass counter blocks
     * (its own included; remote ones mapped over xGMI by IPC), ctr_slot = this pass's block.  With
     * n_peers > 1 bias_func's running counters are the whole job's: the sums of n_scatt and
     * n_recorded and the max of max tau_scatt over the ranks' blocks of this pass. */
    const DevCounters *const *peers;
    int n_peers, ctr_slot;
    /* split_kernel (grm_split.hip): an interaction wave runs its block once split_thr / 64 of its
     * active lanes have a step ready, or after split_spin short sleeps */
    int split_thr, split_spin;
    int split_gthr; /* a geometry wave pushes once split_gthr / 64 of its live lanes can (or after split_spin sleeps) */
    int split_mode; /* 1: waves 0-3 geometry, 4-7 interaction; 2: roles by the SIMD a wave runs on */
    int split_batch; /* consecutive ready slots an interaction lane may evaluate per round */
    /* the early worker's own children (GRM_OPT_EARLY_CHILDREN): a scattering on a pair appends the
     * child's scatter request to the early queue (LoneRec::pad = 1, queue_child_push), where the next
     * free pair sets it up and tracks it (child_setup_body); *early_fin counts the queue slots
     * finished -- tracked, or given up by a pair that left -- and *early_kids the children appended */
    int early_kids_on;
    unsigned long long *early_fin, *early_kids;
    /* the lone kernel's own children (the same option): a scattering on a lone pair appends the child's
     * request to lk_q (lk_tail; published by lk_ready[slot] = lk_tag), which the pairs that have
     * finished their photon take in order (lk_taken); lk_active counts the pairs tracking a photon
     * and lk_standby those waiting for a child (at most LK_STANDBY wait; the rest leave) */
    int lk_on;
    LoneRec *lk_q;
    unsigned long long *lk_ready, lk_cap, lk_tag;
    unsigned long long *lk_tail, *lk_taken, *lk_active, *lk_standby;
    unsigned long long *lk_orig; /* handed-over photons whose pair has finished them */
};
constexpr int STUCK_WORDS = 16, STUCK_CAP = 256;
constexpr unsigned REFRESH_TRIPS = 64; /* counter flush + bias refresh + watchdog period (power of 2) */

/* Per-step (or rarer) lane fields: an LDS column per lane ([field][lane], conflict-free), read and
 * written where used -- what brings the kernel's register demand under the 256 VGPRs two waves per
 * SIMD allow. */
#define GRM_LANE_XFIELDS(X)                                                                          \
    X(tau_abs, 0) X(tau_scatt, 1) X(alpha_scatti, 2) X(alpha_absi, 3) X(bi, 4) X(fl_ne, 5)          \
    X(ph2_e0s, 6)     /* photon_2's e_0_s (its x^1..3, k, dk are in the ph2 LDS slot) */              \
    X(p_dtau_abs, 7) X(p_dtau_scatt, 8) X(p_wc, 9) /* carried across the re-push */
constexpr int LANE_XFIELDS = 10;
#define GRM_LANE_IFIELDS(X)                                                                          \
    X(n_scatt, 0)                                                                                    \
    X(flight, 1) /* warm-up: photons started (+) / ended (-) since the last flush */                \
    /* the lane's launch counters (widened and wave-reduced at exit) */                              \
    X(c_tracked, 2) X(c_primaries, 3) X(c_children, 4) X(c_nstep_max, 5) X(c_long, 6)
constexpr int LANE_IFIELDS = 7;
/* [field][lane], indexed with threadIdx.x so that every access is one ds_read/ds_write_b64 with an
 * immediate offset (a generic pointer here would turn them into FLAT accesses, which also count in
 * vmcnt and cost a 64-bit address register each) */
__shared__ double s_lanex[LANE_XFIELDS * GRM_BLOCK];
/* volatile (the compiler must not keep the fields in registers across trips -- the point is to free
 * them) and typed in the LDS address space (a generic volatile access becomes FLAT + vmcnt waits) */
typedef __attribute__((address_space(3))) volatile double LdsDouble;
__shared__ int s_lanei[LANE_IFIELDS * GRM_BLOCK];
typedef __attribute__((address_space(3))) volatile int LdsInt;

/* hot photon state: lives in VGPRs (and, see above, LDS) for the photon's whole life */
struct Lane {
    double x[4], k[4], dk[4];
    double w, e_0_s;
    int n_step;
    Rng rng;
    /* per-trip push state machine: phase 0 = loop top, 1 = geodesic step in progress,
     * 2 = re-push to the scattering point in progress; depth/pend = position in the halving tree */
    int phase, depth;
    uint32_t pend;
    double dl, hlen;                      /* step size of this iteration; length being pushed */
#define X(name, i) \
    __device__ __forceinline__ LdsDouble &name() const { return ((LdsDouble *)s_lanex)[(i) * GRM_BLOCK + threadIdx.x]; }
#define XI(name, i) \
    __device__ __forceinline__ LdsInt &name() const { return ((LdsInt *)s_lanei)[(i) * GRM_BLOCK + threadIdx.x]; }
    GRM_LANE_XFIELDS(X)
    GRM_LANE_IFIELDS(XI)
#undef X
#undef XI
};

/* Denominator of bias_func's first term, bias_norm * max_tau_scatt * (<N_scatt> + 2)
 * (harm_model.cpp:1391-1404).  Wave-uniform: computed once per refresh at a converged point of the
 * lane loop from the frozen snapshot or from the live device counters -- the live counters sit in
 * device-coherent memory (every XCD adds to them), so loading them per step would put a
 * cross-die round trip on every interaction. */
__device__ __forceinline__ double bias_den(const Params &P, const Ctl &C) {
    double scatt, rec, mts;
    if (C.bias_frozen) {
        scatt = C.f_scatt;
        rec = C.f_rec;
        mts = C.f_maxtau;
    } else if (C.n_peers > 1) {
        /* the job's counters: lane r reads rank r's block of this pass (one remote round trip for
         * the wave, every REFRESH_TRIPS trips), then a wave reduction (converged callers only) */
        const int lane = (int)(threadIdx.x & 63);
        unsigned long long sc = 0, rc = 0, mt = 0;
        if (lane < C.n_peers) {
            const DevCounters *pc = C.peers[lane] + C.ctr_slot;
            sc = __hip_atomic_load(&pc->n_scatt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            rc = __hip_atomic_load(&pc->n_recorded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            mt = __hip_atomic_load(&pc->max_tau_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            sc += __shfl_xor(sc, o);
            rc += __shfl_xor(rc, o);
            mt = max(mt, (unsigned long long)__shfl_xor(mt, o));
        }
        scatt = (double)sc;
        rec = (double)rc;
        mts = __longlong_as_double((long long)mt);
    } else { /* live, reference-like adaptive bias */
        scatt = (double)__hip_atomic_load(&C.ctr->n_scatt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rec = (double)__hip_atomic_load(&C.ctr->n_recorded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mts = __longlong_as_double(
            (long long)__hip_atomic_load(&C.ctr->max_tau_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    const double avg = scatt / (1.0 * rec + 1.0);
    const long long d = __double_as_longlong(P.bias_norm * mts * (avg + 2.0));
    const int lo = __builtin_amdgcn_readfirstlane((int)(d & 0xffffffffll));
    const int hi = __builtin_amdgcn_readfirstlane((int)(d >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

/* The job's warm-up state across ranks (n_peers > 1): photons admitted and photons in flight,
 * summed over the ranks' blocks of this pass (DevCounters::warm; lane r reads rank r's).  A rank
 * whose admission is over no longer counts its flight (its waves stop reporting ends), a rank that
 * has not started the pass reads zero.  Converged callers only. */
__device__ __forceinline__ void warm_job(const Ctl &C, unsigned long long &hist, long long &flight) {
    const int lane = (int)(threadIdx.x & 63);
    unsigned long long h = 0;
    long long f = 0;
    if (lane < C.n_peers) {
        const unsigned long long v =
            __hip_atomic_load(&(C.peers[lane] + C.ctr_slot)->warm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long r = v & ~(WARM_DONE | WARM_STARTED);
        h = (r + (WARM_HIST >> 1)) >> 32; /* flight may be negative between a claim and its undo */
        f = (v & WARM_DONE) ? 0 : (long long)(r - h * WARM_HIST);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        h += __shfl_xor(h, o);
        f += __shfl_xor(f, o);
    }
    hist = h;
    flight = f < 0 ? 0 : f;
}

/* The job's start barrier (n_peers > 1): has every rank's transport launch of this pass started
 * (WARM_STARTED in its pass block)?  A rank that began its warm-up before the others' launches were
 * resident -- a launch queued behind other work, or on the one-GPU emulation behind the other ranks'
 * emission -- would admit the job's first batches alone and run its bulk on a history the job never
 * had.  Converged callers only. */
__device__ __forceinline__ bool job_started(const Ctl &C) {
    const int lane = (int)(threadIdx.x & 63);
    bool ok = true;
    if (lane < C.n_peers)
        ok = (__hip_atomic_load(&(C.peers[lane] + C.ctr_slot)->warm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) &
              WARM_STARTED) != 0;
    return __ballot(!ok) == 0;
}

/* bias_func (harm_model.cpp:1391-1404), same expression and rounding as the reference */
__device__ __forceinline__ double bias_func(double den, double t_e, double w) {
    /* the constant divisions as multiplications by the rounded reciprocal (<= 1 ulp; an IEEE divide
     * is 11 VALU ops and these run every step) */
    const double max = w * (0.5 / WEIGHT_MIN);
    double bias = fdiv(100.0 * t_e * t_e, den);
    if (bias < TP_OVER_TE) bias = TP_OVER_TE;
    if (bias > max) bias = max;
    return bias * (1.0 / TP_OVER_TE);
}

/* Diagnostic build (-DGRM_TIMING): per-wave cycle attribution with s_memtime stamps, accumulated in
 * LDS by the first active lane.  Slots: 0 child refill+sampling, 1 pool refill+init, 2 transport
 * trip, 3 loop total, 4 trips, 5 trips with a child sampled, 6 trips with an init, 7 bias refresh,
 * 8 phase-0 block, 9 push attempt, 10 restore / halving bookkeeping, 11 fluid gather,
 * 12 radiation + bias, 13 rest of the interaction, 14 refill decision and claims (the loop top to
 * the refill loads); 15 = last stamp.  Never built into the product. */
#ifdef GRM_TIMING
__shared__ unsigned long long g_tlds[GRM_BLOCK / 64][24];
__device__ __forceinline__ void tstamp(int r) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long ex = __ballot(1);
    const int w = threadIdx.x >> 6;
    if ((int)(threadIdx.x & 63) == __ffsll((long long)ex) - 1) {
        g_tlds[w][r] += t - g_tlds[w][15];
        g_tlds[w][15] = t;
    }
}
#define TSTAMP(r) tstamp(r)
#define TCOUNT(r) do { if ((threadIdx.x & 63) == 0) g_tlds[threadIdx.x >> 6][r] += 1; } while (0)
/* lane occupancy of a block: slot r counts executions, r + 1 the lanes in them (divergent callers) */
#define TLANES(r, pred)                                                                            \
    do {                                                                                           \
        const unsigned long long b_ = __ballot(pred);                                              \
        if (b_ && (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) {               \
            g_tlds[threadIdx.x >> 6][r] += 1;                                                      \
            g_tlds[threadIdx.x >> 6][(r) + 1] += __popcll(b_);                                     \
        }                                                                                          \
    } while (0)
#else
#define TSTAMP(r) do { } while (0)
#define TCOUNT(r) do { } while (0)
#define TLANES(r, pred) do { } while (0)
#endif

/* stop_criterion (harm_model.cpp:1589-1616) */
__device__ __forceinline__ bool stop_criterion(const Params &P, double x1, double &w, Rng &rng) {
    if (x1 < P.x1_min) return true;
    if (x1 > P.x1_max) {
        if (w < WEIGHT_MIN) {
            if (uniform(rng) <= 1.0 / ROULETTE)
                w *= ROULETTE;
            else
                w = 0.0;
        }
        return true;
    }
    if (w < WEIGHT_MIN) {
        if (uniform(rng) <= 1.0 / ROULETTE) {
            w *= ROULETTE;
        } else {
            w = 0.0;
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ bool stop_criterion(const Params &P, Lane &L) { return stop_criterion(P, L.x[1], L.w, L.rng); }

__device__ void write_trace(const Ctl &C, const Cold *cold, uint64_t id, double w, double x1, double x2,
                                         double x3, double tau_abs, double tau_scatt, int n_scatt, int n_step,
                                         int reason, int ix2, int i_e) {
    const unsigned long long t = atomicAdd(C.trace_count, 1ull);
    if (t >= C.trace_cap) return;
    grm_trace &r = C.trace[t];
    r.id = id;
    r.parent_id = cold ? cold->parent : ~0ull;
    r.w = w;
    r.e = cold ? cold->e : 0.0;
    r.x1 = x1;
    r.x2 = x2;
    r.x3 = x3;
    r.tau_abs = tau_abs;
    r.tau_scatt = tau_scatt;
    r.n_scatt = n_scatt;
    r.n_step = n_step;
    r.end_reason = reason;
    r.ix2 = ix2;
    r.i_e = i_e;
    r.pad_ = 0;
}

__device__ __forceinline__ void trace_end(const Ctl &C, const Cold *cold, const Lane &L, int reason) {
    if (C.trace)
        write_trace(C, cold, L.rng.id, L.w, L.x[1], L.x[2], L.x[3], L.tau_abs(), L.tau_scatt(), L.n_scatt(), L.n_step,
                    reason, -1, -1);
}

/* Workgroup-private spectrum slice in HBM and per-wave counter deltas in LDS.  The block adds its
 * slice to the global spectrum once, at exit; counter deltas are flushed by each wave at its
 * bias-refresh points.  Field f of a cell = field f of grm_spectrum_cell (e_0, never accumulated, is
 * left out); a slice cell is padded to 16 doubles = 128 B, so one record's twelve adds are two
 * aligned 64-B segments.
 *
 * Records are not added one by one.  An fp64 atomic add executes at the memory side (it leaves L2
 * as a 64-B request, MI355X_MICROARCH.md "Global float atomics"), and a no-return atomic stays
 * counted in vmcnt for ~1-3 k cycles: a record's twelve single-lane atomics cost twelve fabric
 * requests, and the wave's next wait for a load of its own (the zone gather) waited for them too.
 * record_super_photon here writes the record's twelve addends into a per-wave LDS buffer
 * (RECBUF_N records); at a converged point of the lane loop a wave with RECBUF_FLUSH or more
 * buffered records adds them with the whole wave, one lane per (record, field): 16 records in 3
 * wave-instructions, ~2 requests per record.  A buffer found full falls back to the direct adds. */
constexpr int SPEC_FIELDS = 12;
constexpr int SPEC_CELL = 16;                              /* padded slice cell (doubles) */
constexpr int SPEC_LDS = N_TH_BINS * N_E_BINS * SPEC_CELL; /* doubles per slice */
__device__ __forceinline__ double *spec_slice(const Ctl &C) { return C.spec_blocks + (size_t)blockIdx.x * SPEC_LDS; }
constexpr int RECBUF_N = 16, RECBUF_FLUSH = 8;
/* the waves that record (all of a track_kernel / lone workgroup; the interaction waves of the split
 * kernel, grm_split.hip) and a wave's index among them */
#ifndef GRM_REC_WAVES
#define GRM_REC_WAVES (GRM_BLOCK / 64)
#define GRM_REC_WAVE(t) ((t) >> 6)
#endif
__shared__ double s_recv[GRM_REC_WAVES][RECBUF_N * SPEC_FIELDS]; /* per-wave record addends */
__shared__ int s_recc[GRM_REC_WAVES][RECBUF_N];                   /* their slice cells */
__shared__ int s_recn[GRM_REC_WAVES];                             /* records buffered */
__shared__ unsigned long long s_cnt[GRM_REC_WAVES][4]; /* n_recorded, n_scatt, max tau bits, max flushed */

__device__ __forceinline__ void flush_counters(const Ctl &C) {
    if ((threadIdx.x & 63) == 0) {
        unsigned long long *c = s_cnt[GRM_REC_WAVE(threadIdx.x)];
        if (c[0]) {
            atomicAdd(&C.ctr->n_recorded, c[0]);
            c[0] = 0;
        }
        if (c[1]) {
            atomicAdd(&C.ctr->n_scatt, c[1]);
            c[1] = 0;
        }
        if (c[2] > c[3]) {
            atomicMax(&C.ctr->max_tau_bits, c[2]);
            c[3] = c[2];
        }
    }
}

/* record_super_photon (harm_model.cpp:1291-1335).  cell_stride == SPEC_CELL: into the wave's record
 * buffer (track_kernel; spec = the workgroup's slice for the fallback); else twelve direct adds
 * into spec (the global spectrum, lone / early kernels) */
__device__ void record_photon(const Params &P, const Ctl &C, const Cold *cold, uint64_t id, double w, double x1,
                              double x2, double x3, double tau_abs, double tau_scatt, int n_scatt, int n_step,
                              double *spec, int cell_stride) {
    int ix2 = -1, i_e = -1, reason = 1;
    const double e = cold->e;
    if (!(isnan(w) || isnan(e))) {
        unsigned long long *cnt = s_cnt[GRM_REC_WAVE(threadIdx.x)];
        atomicMax(cnt + 2, (unsigned long long)__double_as_longlong(tau_scatt)); /* tau_scatt >= 0 */
        if (x2 < 0.5 * (P.xs2 + P.xe2))
            ix2 = (int)(x2 / P.th_dx2);
        else
            ix2 = (int)((P.xe2 - x2) / P.th_dx2);
        if (ix2 >= 0 && ix2 < N_TH_BINS) {
            i_e = (int)((flog(e) - P.spec_l_e_0) / SPEC_D_L_E + 2.5) - 2;
            if (i_e >= 0 && i_e < N_E_BINS) {
                reason = 0;
                atomicAdd(cnt + 0, 1ull);
                atomicAdd(cnt + 1, (unsigned long long)n_scatt);
                const int cell = ix2 * N_E_BINS + i_e;
                double *s = spec + cell * cell_stride;
                const double x1i = cold->x1i, x2i = cold->x2i;
                int slot = RECBUF_N;
                if (cell_stride == SPEC_CELL) {
                    const int wv = GRM_REC_WAVE(threadIdx.x);
                    slot = atomicAdd(&s_recn[wv], 1);
                    if (slot < RECBUF_N) {
                        double *b = &s_recv[wv][slot * SPEC_FIELDS];
                        b[0] = w;
                        b[1] = w * e;
                        b[2] = 1.0;
                        b[3] = (double)n_scatt;
                        b[4] = w * x1i;
                        b[5] = w * (x2i * x2i);
                        b[6] = w * (x3 * x3);
                        b[7] = w * tau_abs;
                        b[8] = w * tau_scatt;
                        b[9] = w * cold->n_e_0;
                        b[10] = w * cold->theta_e_0;
                        b[11] = w * cold->b_0;
                        s_recc[wv][slot] = cell;
                    }
                }
                if (slot >= RECBUF_N) {
                atomicAdd(s + 0, w);                      /* dn_dle */
                atomicAdd(s + 1, w * e);                  /* de_dle */
                atomicAdd(s + 2, 1.0);                    /* nph */
                atomicAdd(s + 3, (double)n_scatt);        /* nscatt */
                atomicAdd(s + 4, w * x1i);                /* x1i_av */
                atomicAdd(s + 5, w * (x2i * x2i));        /* x2i_sq */
                atomicAdd(s + 6, w * (x3 * x3));          /* x3f_sq */
                atomicAdd(s + 7, w * tau_abs);            /* tau_abs */
                atomicAdd(s + 8, w * tau_scatt);          /* tau_scatt */
                atomicAdd(s + 9, w * cold->n_e_0);        /* ne_0 */
                atomicAdd(s + 10, w * cold->theta_e_0);   /* theta_e_0 */
                atomicAdd(s + 11, w * cold->b_0);         /* b_0 */
                }
            } else {
                i_e = -1;
            }
        } else {
            ix2 = -1;
        }
    }
    if (C.trace)
        write_trace(C, cold, id, w, x1, x2, x3, tau_abs, tau_scatt, n_scatt, n_step, reason, ix2, i_e);
}

__device__ __forceinline__ void end_of_life(const Params &P, const Ctl &C, const Cold *cold, const Lane &L) {
    /* record_criterion (harm_model.cpp:1618) && n_step <= max_n_step (:1066) */
    if (L.x[1] > P.x1_max && L.n_step <= MAX_N_STEP)
        record_photon(P, C, cold, L.rng.id, L.w, L.x[1], L.x[2], L.x[3], L.tau_abs(), L.tau_scatt(), L.n_scatt(), L.n_step,
                      spec_slice(C), SPEC_CELL);
    else
        trace_end(C, cold, L, 2);
}

/* the wave's buffered records into the workgroup's slice: lane j adds field j % 12 of record j / 12
 * (called by the whole wave at a converged point) */
__device__ __forceinline__ void flush_records(const Ctl &C) {
    const int wv = GRM_REC_WAVE(threadIdx.x), lane = threadIdx.x & 63;
    const int n = min(__builtin_amdgcn_readfirstlane(s_recn[wv]), RECBUF_N);
    double *slice = spec_slice(C);
    for (int j = lane; j < n * SPEC_FIELDS; j += 64) {
        const int r = j / SPEC_FIELDS, f = j - r * SPEC_FIELDS;
        atomicAdd(slice + s_recc[wv][r] * SPEC_CELL + f, s_recv[wv][j]);
    }
    if (lane == 0) s_recn[wv] = 0;
}

/* emitted photon -> lane (harm_model.cpp:373-391); n_scatt = 0 is the caller's */
__device__ __forceinline__ void load_primary_core(const Ctl &C, uint64_t idx, Rng &rng, double x[4], double k[4],
                                                  double &w, Cold *cold) {
    const double2 *s = reinterpret_cast<const double2 *>(reinterpret_cast<const grm_init_photon *>(C.pool) + idx);
    double2 v[7]; /* x, k, w, e, l, n_e_0, theta_e_0, b_0 (e_0 and n_scatt = 0 are not needed) */
#pragma unroll
    for (int q = 0; q < 7; ++q) v[q] = s[q];
    x[0] = v[0].x; x[1] = v[0].y; x[2] = v[1].x; x[3] = v[1].y;
    k[0] = v[2].x; k[1] = v[2].y; k[2] = v[3].x; k[3] = v[3].y;
    w = v[4].x;
    rng.id = C.id_base + idx;
    rng.ctr = 0;
    rng.ctr_hi = 0;
    Cold c;
    c.e = v[4].y;
    c.x1i = x[1];
    c.x2i = x[2];
    c.n_e_0 = v[5].y;
    c.theta_e_0 = v[6].x;
    c.b_0 = v[6].y;
    c.parent = ~0ull;
    c.pad = 0.0;
    *cold = c;
}

__device__ __forceinline__ void load_primary(const Ctl &C, uint64_t idx, Lane &L, Cold *cold) {
    load_primary_core(C, idx, L.rng, L.x, L.k, L.w, cold);
    L.n_scatt() = 0;
}

/* scatter request -> child photon in the lane (scatter_super_photon after its first
 * validity check, harm_model.cpp:1083-1144, with sample_scattered_photon :1147-1215).
 * false = child invalid (k_tetrad out of range or NaN). */
__device__ __forceinline__ bool sample_child_core(const Params &P, const SReq &R, Rng &rng, double x[4], double k[4],
                                                  double &w, Cold *cold) {
    rng.id = R.id;
    rng.ctr = 0;
    rng.ctr_hi = 0;
    w = R.w;
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = R.x[i];
    Cold c;
    c.x1i = R.x[1];
    c.x2i = R.x[2];
    c.n_e_0 = R.n_e_0;
    c.theta_e_0 = R.theta_e_0;
    c.b_0 = R.b;
    c.parent = R.parent;
    c.e = 0.0;
    c.pad = 0.0;
    Trig T;
    trig_at(P, R.x, T);
    Gcov G;
    gcov_from_trig(P, T, G);
    double bh[4];
    if (R.b > 0.0) {
        const double s = R.b / P.b_unit;
#pragma unroll
        for (int i = 0; i < 4; ++i) bh[i] = R.b_con[i] / s;
    } else {
        bh[0] = 0.0; bh[1] = 1.0; bh[2] = 0.0; bh[3] = 0.0;
    }
    double ec[4][4];
    make_tetrad(R.u_con, bh, G, ec);
    double kt[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double el[4];
        tetrad_cov_row(ec, G, i, el);
        kt[i] = el[0] * R.k[0] + el[1] * R.k[1] + el[2] * R.k[2] + el[3] * R.k[3];
    }
    bool ok = !(kt[0] > 1.0e5 || kt[0] < 0.0 || isnan(kt[1]));
    if (ok) {
        double p[4], ktp[4];
        sample_electron(rng, kt, p, R.theta_e);
        sample_scattered(rng, kt, p, ktp);
#pragma unroll
        for (int i = 0; i < 4; ++i) k[i] = ec[0][i] * ktp[0] + ec[1][i] * ktp[1] + ec[2][i] * ktp[2] + ec[3][i] * ktp[3];
        ok = !isnan(k[1]);
        if (ok) {
            /* e_cov^T (-k0', k1', k2', k3'): only component 0 is needed (e; l enters no result) */
            ktp[0] = -ktp[0];
            double t0 = 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double el[4];
                tetrad_cov_row(ec, G, j, el);
                t0 += el[0] * ktp[j];
            }
            c.e = -t0;
        }
    }
    *cold = c;
    return ok;
}

__device__ bool sample_child(const Params &P, const Ctl &C, const SReq &R, Lane &L, Cold *cold) {
    L.n_scatt() = R.n_scatt;
    return sample_child_core(P, R, L.rng, L.x, L.k, L.w, cold);
}

__device__ __forceinline__ void load_sreq(const SReq *src, SReq &R) {
    const double2 *s = reinterpret_cast<const double2 *>(src);
    double2 *d = reinterpret_cast<double2 *>(&R);
#pragma unroll
    for (int q = 0; q < 12; ++q) d[q] = s[q];
}

__device__ __forceinline__ void store_sreq(SReq *dst, const SReq &R) {
    const double2 *s = reinterpret_cast<const double2 *>(&R);
    double2 *d = reinterpret_cast<double2 *>(dst);
#pragma unroll
    for (int q = 0; q < 12; ++q) d[q] = s[q];
}

/* the scatter request of a scattered photon's child (scatter_super_photon's inputs, :1071-1145) */
__device__ __forceinline__ void make_sreq(SReq &R, const double x[4], const double k[4], const Rng &rng, int n_scatt,
                                          const Cold *cold, const Fluid &F, double wc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        /* x^0 (Boyer-Lindquist time) enters no result -- not the metric (stationary), the fluid, the
         * record or any test -- so the device does not carry it: children start at x^0 = 0 */
        R.x[i] = i == 0 ? 0.0 : x[i];
        R.k[i] = k[i];
        R.u_con[i] = F.u_con[i];
        R.b_con[i] = F.b_con[i];
    }
    R.b = F.b;
    R.theta_e = F.theta_e;
    R.w = wc;
    R.n_e_0 = cold->n_e_0;
    R.theta_e_0 = cold->theta_e_0;
    R.id = child_id(rng.id, rng.ctr);
    R.parent = rng.id;
    R.n_scatt = n_scatt + 1;
    R.pad0 = 0;
}

/* append to the overflow pool (tracked by the next launch) */
__device__ __forceinline__ void push_overflow_req(const Ctl &C, const SReq &R) {
    const unsigned long long o = atomicAdd(C.ovf_count, 1ull);
    if (o < C.ovf_cap)
        store_sreq(C.ovf + o, R);
    else
        atomicAdd(&C.ctr->n_dropped, 1ull);
    atomicAdd(&C.ctr->n_overflow, 1ull);
}

/* push the scattered photon's child out as a scatter request: onto the wave's stack (HBM entries,
 * top counter in LDS), else the overflow pool (tracked by the next launch).  true = on the stack */
__device__ __forceinline__ bool push_request(const Ctl &C, const double x[4], const double k[4], const Rng &rng,
                                             int n_scatt, const Cold *cold, const Fluid &F, double wc, SReq *wstack,
                                             int *wtop) {
    SReq R;
    make_sreq(R, x, k, rng, n_scatt, cold, F, wc);
    const int slot = atomicAdd(wtop, 1); /* LDS; values past the cap are clamped at the next refill */
    if (slot < WSTACK_CAP) {
        store_sreq(wstack + slot, R);
        return true;
    }
    push_overflow_req(C, R);
    return false;
}

/* Two per-lane state copies live in LDS ([slot][lane], conflict-free 8-B words), 11 slots each:
 * x^1..x^3, k, dk/dlambda; photon_2's e_0_s is a lane field.
 *   ph2: photon_2 (harm_model.cpp:920-925), also the depth-0 backup of push_photon;
 *   bk:  the backup of push_photon at depth > 0 (x_cpy/k_cpy/dk_cpy, :1222-1228).
 * 2 x 11 x 8 B x 512 lanes = 88 KB (+ 40 KB of lane fields, 16 KB of lane ints): no global memory
 * traffic on the halving path. */
constexpr int LDS_DOUBLES_PER_LANE = 11;
#ifndef GRM_WARM_BLOCKS
#define GRM_WARM_BLOCKS 64
#endif
#ifndef GRM_WARM_WAVES
#define GRM_WARM_WAVES 8
#endif
constexpr unsigned WARM_BLOCKS = GRM_WARM_BLOCKS; /* workgroups that take the warm-up's admission batches */
constexpr unsigned WARM_WAVES = GRM_WARM_WAVES;   /* ... and their waves that do (waves 0-3: one per SIMD) */
constexpr unsigned PHASE_LOG = 64;   /* words of the launch's phase log (after the per-wave record) */
constexpr unsigned long long RES_CHUNK = 64; /* claim positions a wave reserves per pool-head atomic */
/* The launch-control words (grm_engine::d_small: pool head, in-flight, admission end, hand-over and
 * early-worker words) one per SMALL_STRIDE words, each in a cache line of its own: the warm-up's
 * CAS / atomics on the pool head and the in-flight count, the parked waves' polls of the admission
 * end and the early worker's queue words would otherwise all queue on one 128-B line */
#ifndef GRM_SMALL_STRIDE
#define GRM_SMALL_STRIDE 32
#endif
constexpr int SMALL_STRIDE = GRM_SMALL_STRIDE;
/* waves parked during the warm-up poll the admission end once per PARK_SLEEPS x s_sleep(127) */
#ifndef GRM_PARK_SLEEPS
#define GRM_PARK_SLEEPS 1
#endif

__device__ __forceinline__ void save_xkdk(const Slot &s, const Lane &L) {
#pragma unroll
    for (int i = 0; i < 3; ++i) s[i] = L.x[1 + i];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s[3 + i] = L.k[i];
        s[7 + i] = L.dk[i];
    }
}

__device__ __forceinline__ void load_xkdk(const Slot &s, Lane &L) {
#pragma unroll
    for (int i = 0; i < 3; ++i) L.x[1 + i] = s[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        L.k[i] = s[3 + i];
        L.dk[i] = s[7 + i];
    }
}

__device__ __forceinline__ void store_ph2(const Slot &ph2, Lane &L) {
    L.ph2_e0s() = L.e_0_s;
    save_xkdk(ph2, L);
}

__device__ __forceinline__ void load_ph2(const Slot &ph2, Lane &L) {
    load_xkdk(ph2, L);
}

/* photon set-up at the head of track_super_photon (harm_model.cpp:895-917).  Here only the validity
 * check and the counters; the rest -- fluid and absorption/scattering coefficients at x, bias, and
 * dk/dlambda from the connection at x (init_dkdlam) -- runs on the lane's next trip as phase 3,
 * inside the same push and fluid/radiation code the stepping lanes execute (see transport_trip), so
 * a refill costs a few loads instead of a divergent block of its own.  false = invalid. */
__device__ bool init_photon(const Ctl &C, const Cold *cold, Lane &L, const Slot &ph2) {
    if (isnan(L.x[0]) || isnan(L.x[1]) || isnan(L.x[2]) || isnan(L.x[3]) || isnan(L.k[0]) || isnan(L.k[1]) ||
        isnan(L.k[2]) || isnan(L.k[3]) || L.w == 0.0) {
        L.n_step = 0; /* the trace record is this photon's, not the lane's last one */
        L.tau_abs() = L.tau_scatt() = 0.0;
        trace_end(C, cold, L, 4);
        return false;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) L.dk[i] = 0.0;
    store_ph2(ph2, L); /* x, k kept here across the set-up's zero-length push */
    L.n_step = 0;
    L.tau_abs() = L.tau_scatt() = 0.0;
    L.e_0_s = cold->e;
    L.hlen = 0.0;
    L.depth = 0;
    L.pend = 0;
    L.phase = 3;
    return true;
}

/* Head of a geodesic step (phase 0): stop test, photon_2, step size (harm_model.cpp:919-927).
 * false = the photon's life ended. */
__device__ __forceinline__ bool trip_begin(const Params &P, const Ctl &C, Lane &L, Cold *cold, const Slot &ph2) {
    if (stop_criterion(P, L)) {
        end_of_life(P, C, cold, L);
        return false;
    }
    /* photon_2 (:920-925) -- also the depth-0 backup of the push */
    store_ph2(ph2, L);
    L.dl = step_size(P, L.x, L.k);
    L.hlen = L.dl;
    L.depth = 0;
    L.pend = 0;
    L.phase = 1;
    return true;
}

/* lane `src`'s value of v (src wave-uniform) */
__device__ __forceinline__ double bcast(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, src), hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

/* Tail speculation.  A wave whose only work left is ONE photon (the pool is drained and its stack
 * empty) completes that photon's current push -- push_photon's halving recursion,
 * harm_model.cpp:1217-1289 -- with all its lanes: from the start state of every sub-step the owner
 * attempts depth d and idle lane r attempts depth d + r, at once.  The serial walk would attempt d,
 * then (restored to the same start state) d + 1, ... until one passes or depth MAX_SUBDIV accepts
 * whatever it gets; each of these attempts is made here from bit-identical inputs, so the shallowest
 * accepted one IS the serial walk's sub-step, its failed shallower attempts become the pending
 * second halves they would have left, and the walk goes on from the accepted state.  One round per
 * accepted sub-step instead of one trip per attempt: the photons that halve to depth 7 on every
 * step (255 attempts for 128 sub-steps) -- the last photons of a pass -- run ~2x faster.
 * Called by the whole wave (converged); `owner` is wave-uniform.  Every lane's copy of the push
 * state (x, k, dk/dlambda, e_0_s, hlen, depth, pend) follows the owner's; only the owner's is used. */
/* The halving walk proper, on a push state every lane of the wave holds identically (x, k, dk/dlambda,
 * e_0_s; the node `depth` of the halving tree being pushed, the pending second halves `pend`); lane
 * rank r (0 for the state's owner) attempts depth + r.  Leaves the completed push in every lane. */
/* QUAD: the lone geometry wave's form -- quad r of lanes attempts depth + r with the quad-parallel
 * push (push_attempt_quad), rank = lane / 4 (16 ranks still cover every depth to MAX_SUBDIV) */
template <bool QUAD = false>
__device__ __forceinline__ int walk_push(const Params &P, double x[4], double k[4], double dk[4], double &e_0_s,
                                         double hlen, int depth, uint32_t pend, int rank, int owner) {
    int rounds = 0; /* attempt rounds (diagnostics) */
    while (true) {
        if (!(x[1] < P.xs1) && depth == MAX_SUBDIV) {
            /* a leaf of the deepest level is accepted whatever its checks say (:1279): every lane makes
             * that one attempt from the identical state, so no lane has to win and be broadcast (the
             * second halves at depth MAX_SUBDIV -- every other round of a photon that halves to full
             * depth, seed 124's tail in round 4) */
            double e_1;
            Trig T;
            Gcov G;
            if (QUAD)
                push_attempt_quad(P, x, k, dk, e_0_s, ldexp(hlen, -MAX_SUBDIV), e_1, T, G, (int)(threadIdx.x & 3));
            else
                push_attempt(P, x, k, dk, e_0_s, ldexp(hlen, -MAX_SUBDIV), e_1, T, G);
            e_0_s = e_1;
            ++rounds;
        } else if (!(x[1] < P.xs1)) {
            /* every lane attempts in place from the same start state; the winner's result is then
             * broadcast over all of them */
            const int d = depth + rank;
            double e_1 = 0.0;
            bool ok = false;
            if (d <= MAX_SUBDIV) {
                Trig T;
                Gcov G;
                const bool fail = QUAD ? push_attempt_quad(P, x, k, dk, e_0_s, ldexp(hlen, -d), e_1, T, G,
                                                              (int)(threadIdx.x & 3))
                                       : push_attempt(P, x, k, dk, e_0_s, ldexp(hlen, -d), e_1, T, G);
                ok = !fail || d == MAX_SUBDIV;
            }
            /* the owner's attempt if it passed, else the shallowest passing helper (helper depth grows
             * with lane index); some lane passes, since 63 helpers cover every depth to MAX_SUBDIV */
            const unsigned long long acc = __ballot(ok);
            ++rounds;
            const int w = ((acc >> owner) & 1ull) ? owner : __ffsll((long long)acc) - 1;
            const int dw = __builtin_amdgcn_readlane(d, w);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                x[i] = bcast(x[i], w);
                k[i] = bcast(k[i], w);
                dk[i] = bcast(dk[i], w);
            }
            e_0_s = bcast(e_1, w);
            pend |= ((2u << dw) - 1u) & ~((2u << depth) - 1u); /* second halves at depths depth+1..dw */
            depth = dw;
        }
        if (pend == 0) break;
        depth = 31 - __builtin_clz(pend);
        pend &= ~(1u << depth);
    }
    return rounds;
}

__device__ __forceinline__ int walk_rank(int owner) {
    const int lane = (int)(threadIdx.x & 63);
    return lane == owner ? 0 : (lane < owner ? lane + 1 : lane);
}

/* complete the owner's push in progress (phase 1 or 2, any node of its halving tree) with the wave */
__device__ __forceinline__ void halving_walk(const Params &P, Lane &L, int owner) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        L.x[i] = bcast(L.x[i], owner);
        L.k[i] = bcast(L.k[i], owner);
        L.dk[i] = bcast(L.dk[i], owner);
    }
    L.e_0_s = bcast(L.e_0_s, owner);
    const double hlen = bcast(L.hlen, owner);
    const int depth = __builtin_amdgcn_readlane(L.depth, owner);
    const uint32_t pend = (uint32_t)__builtin_amdgcn_readlane((int)L.pend, owner);
    walk_push(P, L.x, L.k, L.dk, L.e_0_s, hlen, depth, pend, walk_rank(owner), owner);
    L.depth = 0;
    L.pend = 0;
}

/* Lone photons.  When a wave's only work left is one photon (the pool is drained, its stack empty),
 * that photon's latency is the pass's tail: such photons run for 1e5-1e6 steps (trapped
 * near-circular orbits, polar Zeno stepping, full-depth halving -- all exact reference semantics,
 * which end them only at max_n_step, harm_model.cpp:1058-1063).  The lane loop is the wrong place
 * for them (one lane of 64 busy, per-trip refill logic, lane fields in LDS): the wave hands the
 * photon over (export_lone, at the top of a step) and exits, and after the launch lone_kernel runs
 * every handed-over photon with a whole wave of its own: straight-line steps of
 * track_super_photon's loop (:919-1063) with the state in registers, every lane holding the same
 * values, the pushes as halving walks over the lanes (walk_push), only lane 0 writing.  Its
 * scattered children go to the overflow pool, which the host relaunches the lane loop over. */
struct alignas(16) LoneRec {
    double x[4], k[4], dk[4];
    double w, e_0_s;
    double tau_abs, tau_scatt, a_si, a_ai, bi, fl_ne;
    Cold c;
    uint64_t id;
    uint32_t ctr;
    int32_t n_step, n_scatt, pad;
};
static_assert(sizeof(LoneRec) == 256, "LoneRec layout");
static_assert(sizeof(SReq) <= offsetof(LoneRec, pad), "an early-queue slot holds a scatter request below its pad word");

__device__ __forceinline__ void export_lone(LoneRec *r, const Lane &L, const Cold *cold) {
    /* field by field (a LoneRec built in registers first would add 68 VGPRs at this point of the loop) */
    double2 *d = reinterpret_cast<double2 *>(r);
    d[0] = make_double2(L.x[0], L.x[1]);
    d[1] = make_double2(L.x[2], L.x[3]);
    d[2] = make_double2(L.k[0], L.k[1]);
    d[3] = make_double2(L.k[2], L.k[3]);
    d[4] = make_double2(L.dk[0], L.dk[1]);
    d[5] = make_double2(L.dk[2], L.dk[3]);
    d[6] = make_double2(L.w, L.e_0_s);
    d[7] = make_double2(L.tau_abs(), L.tau_scatt());
    d[8] = make_double2(L.alpha_scatti(), L.alpha_absi());
    d[9] = make_double2(L.bi(), L.fl_ne());
    const double2 *c = reinterpret_cast<const double2 *>(cold);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[10 + q] = c[q];
    r->id = L.rng.id;
    r->ctr = L.rng.ctr;
    r->n_step = L.n_step;
    r->n_scatt = L.n_scatt();
    r->pad = 0;
}

/* the child of a lone photon's scattering, straight to the overflow pool */
__device__ __forceinline__ void push_overflow(const Ctl &C, const double x[4], const double k[4], const Rng &rng,
                                              int n_scatt, const Cold *cold, const Fluid &F, double wc) {
    SReq R;
    make_sreq(R, x, k, rng, n_scatt, cold, F, wc);
    push_overflow_req(C, R);
}

/* the child of an early-worker photon's scattering (lane 0): its scatter request goes into a slot of
 * the early queue, marked as a request (LoneRec::pad = 1; the SReq fills the slot's first 192 B), and
 * the next free pair of the worker sets it up and tracks it at once (child_setup_body), as the
 * reference tracks a child as soon as it is made (harm_model.cpp:1016-1023); the overflow pool when
 * the queue is full.  A slot claimed past the cap is never published, as in the lane loop's
 * hand-over. */
/* kids: 1 the early worker's queue, 2 the lone kernel's (lk_q; its slots are all requests) */
__device__ __forceinline__ void queue_child_push(const Ctl &C, int kids, const double x[4], const double k[4],
                                                 const Rng &rng, int n_scatt, const Cold *cold, const Fluid &F,
                                                 double wc) {
    SReq R;
    make_sreq(R, x, k, rng, n_scatt, cold, F, wc);
    LoneRec *q = kids == 1 ? C.early_q : C.lk_q;
    unsigned long long *ready = kids == 1 ? C.early_ready : C.lk_ready;
    unsigned long long *tail = kids == 1 ? C.early_tail : C.lk_tail;
    const unsigned long long cap = kids == 1 ? C.early_cap : C.lk_cap, tag = kids == 1 ? C.early_tag : C.lk_tag;
    if (__hip_atomic_load(tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cap) {
        const unsigned long long slot = atomicAdd(tail, 1ull);
        if (slot < cap) {
            LoneRec *r = q + slot;
            store_sreq(reinterpret_cast<SReq *>(r), R);
            r->pad = 1;
            if (kids == 1) atomicAdd(C.early_kids, 1ull);
            __threadfence();
            __hip_atomic_store(ready + slot, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    push_overflow_req(C, R);
}

/* Two waves per handed-over photon, pipelined: the geometry wave (wave 1) runs the photon's
 * geodesic ahead -- photon_2, step size, push as a halving walk over its lanes (:920-930) -- into a
 * ring of LONE_RING steps in LDS; the interaction wave (wave 0) consumes them in order and does
 * everything else of the loop body: the stop criteria with their roulette draws, fluid, absorption
 * and scattering coefficients, bias, the scattering decision, the weight (:919, :932-1063).  The
 * geodesic does not depend on the interactions except at a scattering, where the photon continues
 * from photon_2 pushed to the scattering point (:1005-1010): the interaction wave makes that push
 * itself and restarts the geometry wave from it (a new generation; steps of the old one are
 * discarded by their tag).  Both halves of a step then run at once on two SIMDs. */
constexpr int LONE_RING = 32, LONE_BATCH = 16;
constexpr unsigned long long LONE_STOP = ~0ull;
struct alignas(16) LoneSlot {
    double out[13], dl;     /* the state after the push (x, k, dk/dlambda, e_0_s) and the step size */
    unsigned long long tag; /* (generation << 32) | (step index + 1), stored last */
};
struct alignas(16) LoneCtl {
    double rs[13];                /* restart state: photon_2 of the generation's first step */
    unsigned long long cons, req; /* steps consumed; restart request (generation << 32 | step) or LONE_STOP */
};
/* one photon's two-wave pipeline state (a geometry wave + an interaction wave) */
struct LonePair {
    LoneSlot ring[LONE_RING];
    LoneCtl ctl;
};
constexpr int LONE_PAIRS = 2; /* pairs of the concurrent worker (early_kernel: 4 waves, one per SIMD, up to 512 VGPRs) */
/* early_kernel dispatches its geometry waves to s_pair[0] / s_pair[1] by a constant index (one inlined
 * copy per pair): more pairs need more arms there, or a pair's interaction wave waits forever */
static_assert(LONE_PAIRS == 2, "early_kernel's geometry dispatch assumes two pairs");
/* early_kernel waits this long (s_memrealtime, 100 MHz) for the bulk launch to start before it
 * takes the launches for serialised and leaves */
constexpr unsigned long long EARLY_ALONE_TICKS = 100000; /* 1 ms */
__shared__ LonePair s_pair[LONE_PAIRS];

__device__ __forceinline__ void pack13(double *d, const double x[4], const double k[4], const double dk[4],
                                       double e) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        d[i] = x[i];
        d[4 + i] = k[i];
        d[8 + i] = dk[i];
    }
    d[12] = e;
}

__device__ __forceinline__ void unpack13(const double *d, double x[4], double k[4], double dk[4], double &e) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[i] = d[i];
        k[i] = d[4 + i];
        dk[i] = d[8 + i];
    }
    e = d[12];
}

/* A kernel argument read afresh where it is used.  The arguments (Params, Ctl: ~0.7 KB) are
 * loop-invariant, so the compiler loads them once at entry and keeps them live across the persistent
 * loop; they do not fit the SGPR file, and the overflow is spilled into VGPR lanes and read back with
 * v_readlane -- a VALU instruction (plus hazard nops) per use, inside the step.  Passing the argument
 * block through an opaque SGPR copy at the top of each trip makes every use a scalar load from the
 * kernarg segment instead (constant address space: s_load, scalar cache, no VALU issue). */
/* The kernarg segment of track_kernel / lone_kernel / early_kernel, all (Params, Ctl): explicit
 * arguments in order at their ABI alignment, i.e. the layout of this struct.  Two traps: the address
 * of a by-value kernel parameter is NOT the kernarg segment (taking it makes the compiler copy the
 * parameter into private memory), and __builtin_amdgcn_kernarg_segment_ptr() is only meaningful in
 * the kernel itself (in a called function it lowers to null): only the kernel takes the pointer
 * (kargs()).  Used by track_kernel only: in the lone pipeline's serial chain the exposed scalar-load
 * latency costs more than the readlanes (lone probe 1.80 vs 1.63 us/step, profiles/r02q_karg_ab.txt). */
struct KArgs {
    Params P;
    Ctl C;
};
static_assert(offsetof(KArgs, C) == sizeof(Params), "kernarg layout: Ctl follows Params");
typedef const KArgs __attribute__((address_space(4))) KArgsK;
/* call only in the body of a kernel whose explicit arguments are exactly (Params, Ctl) */
__device__ __forceinline__ KArgsK *kargs() { return (KArgsK *)__builtin_amdgcn_kernarg_segment_ptr(); }
/* the kernarg segment through an opaque scalar copy of its pointer: loads through it cannot be
 * hoisted out of the loop the copy is made in */
__device__ __forceinline__ KArgsK *karg_fresh(KArgsK *ka) {
    /* (a non-inlined function receives ka in VGPRs: make it scalar first; a no-op in a kernel) */
    const uint64_t a = (uint64_t)ka;
    KArgsK *k = (KArgsK *)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a));
    asm volatile("" : "+s"(k));
    return k;
}
__device__ __forceinline__ const Params &karg_params(KArgsK *k) { return *(const Params *)&k->P; }
__device__ __forceinline__ const Ctl &karg_ctl(KArgsK *k) { return *(const Ctl *)&k->C; }
/* Guard of the kernarg-segment reads: the words the loop reads through kargs() must be the launch's
 * arguments.  Compares, at the ends and in the middle of both blocks, the segment's words with the
 * by-value parameters (which the compiler reads from the segment by its own ABI).  A layout the
 * struct KArgs does not describe (a compiler or ABI change) makes this fail for every wave, and the
 * launch then exits at once with DevCounters::karg_bad set, which the host turns into an error
 * (run_passes): there is no silent wrong-argument mode.  Wave-uniform (scalar loads only). */
__device__ __forceinline__ bool kargs_check(KArgsK *ka, const Params &P, const Ctl &C) {
    const Params &kp = karg_params(ka);
    const Ctl &kc = karg_ctl(ka);
    bool ok = kp.n1 == P.n1 && kp.n2 == P.n2 && __double_as_longlong(kp.a) == __double_as_longlong(P.a) &&
              __double_as_longlong(kp.bias_norm) == __double_as_longlong(P.bias_norm) && kp.zones == P.zones &&
              kp.k2 == P.k2;
    ok = ok && kc.pool == C.pool && kc.n_pool == C.n_pool && kc.ctr == C.ctr && kc.key0 == C.key0 &&
         kc.spec_blocks == C.spec_blocks && kc.watchdog_ticks == C.watchdog_ticks && kc.lanes == C.lanes + C.karg_test &&
         kc.early_steps == C.early_steps;
    return __builtin_amdgcn_readfirstlane((int)ok) != 0;
}

/* The push's uniform inputs for the geometry wave's loop, held in VGPRs.  The lone kernels take
 * (Params, Ctl) by value; the ~0.7 KB of arguments do not fit the SGPR file next to the interaction
 * wave's code, so the compiler spills them into lanes of a VGPR and reloads each use with a
 * v_readlane (a VALU instruction, plus hazard nops before the SGPR is read): 1,118 such reloads in
 * lone_kernel, dozens of them inside one push.  Copies made lane-varying by an empty asm live in
 * VGPR pairs instead (26 VGPRs of the 512 a single wave per SIMD has) and feed the fp64 VALU
 * directly.  Same values, same operations. */
__device__ __forceinline__ void push_params_vgpr(Params &G) {
    asm volatile("" : "+v"(G.a), "+v"(G.a2), "+v"(G.a3), "+v"(G.a4), "+v"(G.r0), "+v"(G.hs1), "+v"(G.hs1_pi));
    asm volatile("" : "+v"(G.th_fac), "+v"(G.d2k), "+v"(G.m2a), "+v"(G.xe2), "+v"(G.xs1));
}

constexpr bool GEO_QUAD = true; /* the geometry wave pushes with quad-parallel corrector rows (§4.2:
                                   * the plain push 1.41-1.42 us/step against 1.36-1.37, s3e) */

/* The geometry wave of a pair (see above): runs photon after photon -- each begins as a restart
 * request from the interaction wave -- until LONE_STOP. */
__device__ void lone_geometry(const Params &P_, const Ctl &C, int lane, LonePair &pr) {
    Params P = P_;
    push_params_vgpr(P);
    unsigned gen = 0;
    unsigned long long p = 0, cur = 0, cons = 0; /* cons: the last value read of pr.ctl.cons */
    bool spec = false; /* speculate the halving depths on this step's push (the last one halved) */
    double x[4], k[4], dk[4], e_0_s;
    {
        /* a photon starts as a restart (generation, step 0) from its hand-over state in rs */
        unsigned long long r0;
        while ((r0 = __hip_atomic_load(&pr.ctl.req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0)
            __builtin_amdgcn_s_sleep(2);
        if (r0 == LONE_STOP) return;
        cur = r0;
        gen = (unsigned)(r0 >> 32);
        p = r0 & 0xffffffffull;
        cons = p;
        unpack13(pr.ctl.rs, x, k, dk, e_0_s);
    }
    const double *ph2src = pr.ctl.rs; /* where the current step's start state (photon_2) is kept */
#ifdef GRM_TIMING
    unsigned long long g_last = __builtin_amdgcn_s_memtime();
    unsigned long long tg[6] = {0, 0, 0, 0, 0, 0}; /* steps, rounds, walk, step size, rest, halved */
#endif
    while (true) {
        if (p + 1 >= cons + LONE_RING) { /* the slot of step p and that of p - 1 must be consumed */
            cons = __hip_atomic_load(&pr.ctl.cons, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (p + 1 >= cons + LONE_RING) {
#ifdef GRM_TIMING
                const unsigned long long t0 = __builtin_amdgcn_s_memtime();
                __builtin_amdgcn_s_sleep(1); /* the ring is full */
                if (lane == 0) atomicAdd(C.timing + 31, __builtin_amdgcn_s_memtime() - t0);
#else
                __builtin_amdgcn_s_sleep(1); /* the ring is full */
#endif
                if (__hip_atomic_load(&pr.ctl.req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == cur) continue;
            }
        }
        /* the restart request (stop folded in as LONE_STOP): read once per step and looked at
         * after the push, so that its LDS latency hides behind it; a step computed while a
         * restart was pending is dropped (and one published just before a restart carries the
         * old generation's tag, which the interaction wave skips) */
        const unsigned long long req = __hip_atomic_load(&pr.ctl.req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef GRM_TIMING
        const unsigned long long g0 = __builtin_amdgcn_s_memtime();
#endif
        const double dl = step_size(P, x, k);
#ifdef GRM_TIMING
        const unsigned long long g1 = __builtin_amdgcn_s_memtime();
#endif
        /* Most steps pass their first attempt: then every lane makes that same attempt, the
         * state stays identical over the wave and needs no broadcast.  A step that halves
         * continues as a halving walk, and the next step speculates from the start. */
        int rounds = 1;
        {
            if (!spec) {
                bool fail = false;
                if (!(x[1] < P.xs1)) {
                    double e_1;
                    Trig T;
                    Gcov G;
                    /* every quad of lanes makes the attempt, lane q contracting connection row q */
                    fail = GEO_QUAD ? push_attempt_quad(P, x, k, dk, e_0_s, dl, e_1, T, G, lane & 3)
                                    : push_attempt(P, x, k, dk, e_0_s, dl, e_1, T, G);
                    if (fail) { /* depth 0 failed: the serial walk goes on at depth 1 (:1279-1285) */
                        /* from the step's start state, photon_2: the slot published last (or the
                         * generation's restart state) -- no register copy on every step for the ~2 %
                         * that fail (the copy cost ~24 moves per step of the serial chain) */
                        double e_r;
                        unpack13(ph2src, x, k, dk, e_r);
                        rounds += walk_push<GEO_QUAD>(P, x, k, dk, e_0_s, dl, 1, 2u, GEO_QUAD ? lane >> 2 : lane, 0);
                    } else {
                        e_0_s = e_1;
                    }
                }
                spec = fail;
            } else {
                rounds = walk_push<GEO_QUAD>(P, x, k, dk, e_0_s, dl, 0, 0u, GEO_QUAD ? lane >> 2 : lane, 0);
                spec = rounds > 1;
            }
        }
        if (req != cur) {
            if (req == LONE_STOP) {
#ifdef GRM_TIMING
                /* slots 16-21: photons of > 1e5 steps (the tail), 22-27: the others */
                if (lane == 0)
                    for (int r = 0; r < 6; ++r) atomicAdd(C.timing + (tg[0] > 100000 ? 16 : 22) + r, tg[r]);
#endif
                break;
            }
            /* restart from the scattering point (this step, if computed, is on the old geodesic) */
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); /* rs was written before req */
            cur = req;
            gen = (unsigned)(req >> 32);
            p = req & 0xffffffffull;
            cons = p; /* what the interaction wave has consumed when it requests a restart at p */
            unpack13(pr.ctl.rs, x, k, dk, e_0_s);
            ph2src = pr.ctl.rs;
            spec = false;
            continue;
        }
#ifdef GRM_TIMING
        const unsigned long long g2 = __builtin_amdgcn_s_memtime();
        tg[0] += 1;
        tg[1] += (unsigned long long)rounds;
        tg[2] += g2 - g1;
        tg[3] += g1 - g0;
        tg[4] += g0 - g_last;
        tg[5] += spec ? 1ull : 0ull;
        g_last = g2;
#endif
        if (lane == 0) {
            LoneSlot &S = pr.ring[p % LONE_RING];
            pack13(S.out, x, k, dk, e_0_s);
            S.dl = dl;
            /* LDS operations of a wave complete in order: the slot is written before its tag
             * (a compiler barrier keeps the stores in program order; no wait for completion) */
            __asm__ volatile("" ::: "memory");
            __hip_atomic_store(&S.tag, ((unsigned long long)gen << 32) | (p + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        ph2src = pr.ring[p % LONE_RING].out; /* lane 0's stores precede this wave's later loads */
        ++p;
    }
}

/* The draws of a lone photon come from a window of 64 consecutive Philox counters evaluated at once
 * (lane i: counter wbase + i; the same block and bits as uniform(), so the same numbers in the same
 * order): a serial draw is then two v_readlane instead of a 10-round Philox chain. */
__device__ __forceinline__ double lone_draw(Rng &rng, double &win, uint32_t &wbase, int lane) {
    if (rng.ctr - wbase >= 64u) { /* wave-uniform */
        wbase = rng.ctr;
        Rng g = rng;
        g.ctr = wbase + (uint32_t)lane;
        win = uniform(g);
    }
    const double u = bcast(win, (int)(rng.ctr - wbase));
    ++rng.ctr;
    return u;
}

/* stop_criterion (harm_model.cpp:1589-1616) with the windowed draws */
__device__ __forceinline__ bool lone_stop(const Params &P, double x1, double &w, Rng &rng, double &win,
                                          uint32_t &wbase, int lane) {
    if (x1 < P.x1_min) return true;
    if (x1 > P.x1_max) {
        if (w < WEIGHT_MIN) {
            if (lone_draw(rng, win, wbase, lane) <= 1.0 / ROULETTE)
                w *= ROULETTE;
            else
                w = 0.0;
        }
        return true;
    }
    if (w < WEIGHT_MIN) {
        if (lone_draw(rng, win, wbase, lane) <= 1.0 / ROULETTE) {
            w *= ROULETTE;
        } else {
            w = 0.0;
            return true;
        }
    }
    return false;
}

/* The interaction wave of a pair: one handed-over photon, from its record to its end (the
 * geometry wave is started on it with a restart request: generation gen + 1, step 0). */
/* kids: where the photon's scattered children go -- 0 the overflow pool, 1 the early worker's queue,
 * 2 the lone kernel's (queue_child_push) */
__device__ void lone_interact(const Params &P, const Ctl &C, const LoneRec &R, int lane, LonePair &pr, unsigned &gen_io,
                              int kids) {
    double x1 = R.x[1];
    unsigned gen = gen_io + 1;
    if (lane == 0) {
        double x[4], k[4], dk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            x[i] = R.x[i];
            k[i] = R.k[i];
            dk[i] = R.dk[i];
        }
        pack13(pr.ctl.rs, x, k, dk, R.e_0_s); /* the state before step 0 */
        pr.ctl.cons = 0;
        __hip_atomic_store(&pr.ctl.req, (unsigned long long)gen << 32, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const bool own = lane == 0;
    const int rank = lane;
    double w = R.w;
    double tau_abs = R.tau_abs, tau_scatt = R.tau_scatt, a_si = R.a_si, a_ai = R.a_ai, bi = R.bi, fl_ne = R.fl_ne;
    const Cold *cold = &R.c;
    int n_step = R.n_step;
    const int n_scatt = R.n_scatt;
    Rng rng;
    rng.k0 = C.key0;
    rng.k1 = C.key1;
    rng.id = R.id;
    rng.ctr = R.ctr;
    rng.ctr_hi = 0;
    double win = 0.0;
    uint32_t wbase = rng.ctr - 64u; /* empty window */
    double bias_d = bias_den(P, C);
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long steps = 0, children = 0;
    bool ended = false, abandoned = false;
    int reason = -1; /* ended without a record: trace reason */
    unsigned long long gen_start = 0; /* the generation's first step */
    unsigned long long si = 0;        /* index of the next step */
    /* the step whose end state is the photon's state (LONE_STOP: the restart state in rs) */
    unsigned long long cur = LONE_STOP;
    unsigned since = 0; /* steps since the last counter flush / bias refresh / watchdog look */
    bool done = false;
#ifdef GRM_TIMING
    unsigned long long ti[4] = {0, 0, 0, 0}; /* batches, steps in them, batch-evaluation cycles, serial cycles */
#endif
    while (!done) {
        /* A batch: the consecutive steps the geometry wave has ready (at least one, at most
         * LONE_BATCH).  Lane j evaluates step si + j at once: the fluid and the absorption /
         * scattering coefficients at its end point (these depend on the geodesic only), and from
         * them -- taking the previous step's coefficients from lane j - 1, as the serial recurrence
         * has them whenever step j interacts -- its optical depths, the weight factor of a step
         * without scattering and the weight-independent part of bias_func.  The steps then run in
         * order, each taking its lane's values; a scattering discards the rest of the batch (the
         * photon continues elsewhere). */
        if (since >= REFRESH_TRIPS) { /* at a batch boundary, so that bias_d is fixed over a batch */
            since = 0;
            flush_counters(C);
            if (!C.bias_frozen) bias_d = bias_den(P, C);
            if (C.watchdog_ticks) {
                bool stop = __hip_atomic_load(&C.ctr->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (!stop && __builtin_amdgcn_s_memrealtime() - rt_start > C.watchdog_ticks) {
                    stop = true;
                    if (own) __hip_atomic_store(&C.ctr->abort, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (stop) {
                    abandoned = true;
                    break;
                }
            }
        }
        const unsigned long long base = si;
        {
            LoneSlot &S0 = pr.ring[base % LONE_RING];
            const unsigned long long want = ((unsigned long long)gen << 32) | (base + 1);
#ifdef GRM_TIMING
            const unsigned long long tw0 = __builtin_amdgcn_s_memtime();
#endif
            while (__hip_atomic_load(&S0.tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != want)
                __builtin_amdgcn_s_sleep(1);
#ifdef GRM_TIMING
            if (own) atomicAdd(C.timing + 30, __builtin_amdgcn_s_memtime() - tw0);
#endif
        }
        const unsigned long long qj = base + (lane < LONE_BATCH ? lane : 0);
        const bool ready = lane < LONE_BATCH && __hip_atomic_load(&pr.ring[qj % LONE_RING].tag, __ATOMIC_ACQUIRE,
                                                                  __HIP_MEMORY_SCOPE_WORKGROUP) ==
                                                    (((unsigned long long)gen << 32) | (qj + 1));
        const unsigned long long rb = __ballot(ready);
        const int nb = rb == ~0ull ? 64 : __ffsll((long long)~rb) - 1; /* leading run of ready steps (>= 1) */
#ifdef GRM_TIMING
        const unsigned long long tb0 = __builtin_amdgcn_s_memtime();
#endif
        double l_x1, l_ne, l_as = 0.0, l_aa = 0.0, l_dts, l_dta, l_b0, l_fac;
        int l_zero;
        {
            const LoneSlot &Sj = pr.ring[(base + (lane < nb ? lane : 0)) % LONE_RING];
            double xj[4], kj[4], dkj[4], ej;
            unpack13(Sj.out, xj, kj, dkj, ej);
            const double dl = Sj.dl;
            Trig T;
            Gcov G;
            ZoneFetch Z;
            zone_fetch(P, xj, Z);
            trig_at(P, xj, T);
            gcov_from_trig(P, T, G);
            Fluid F;
            fluid_from(P, xj, G, Z, F);
            const double nu = fluid_nu(kj, F);
            l_zero = (nu < 0.0 || F.n_e == 0.0) ? 1 : 0; /* bound_flag (:941-955) or nu < 0 */
            if (!l_zero) radiation_coeffs(P, kj, F, nu, l_as, l_aa);
            l_x1 = xj[1];
            l_ne = F.n_e;
            /* the coefficients the step starts from: the step before's (lane j - 1), or the carried
             * (the shuffles outside the conditional: with lane 0 masked off, lane 1 would read 0) */
            const double up_as = __shfl_up(l_as, 1), up_aa = __shfl_up(l_aa, 1);
            const double p_as = lane == 0 ? a_si : up_as, p_aa = lane == 0 ? a_ai : up_aa;
            if (l_zero) {
                l_dts = 0.5 * p_as * P.d_tau_k * dl;
                l_dta = 0.5 * p_aa * P.d_tau_k * dl;
                l_b0 = 0.0;
            } else {
                l_dts = 0.5 * (p_as + l_as) * P.d_tau_k * dl;
                l_dta = 0.5 * (p_aa + l_aa) * P.d_tau_k * dl;
                /* bias_func up to its weight cap (same operations) */
                l_b0 = fdiv(100.0 * F.theta_e * F.theta_e, bias_d);
                if (l_b0 < TP_OVER_TE) l_b0 = TP_OVER_TE;
            }
            const double d_tau = l_dta + l_dts;
            l_fac = d_tau < 1.0e-3 ? (1.0 - d_tau * (1.0 / 24.0) * (24.0 - d_tau * (12.0 - d_tau * (4.0 - d_tau))))
                                   : fexp(-d_tau);
        }
#ifdef GRM_TIMING
        const unsigned long long tb1 = __builtin_amdgcn_s_memtime();
        ti[0] += 1;
        ti[1] += (unsigned long long)nb;
        ti[2] += tb1 - tb0;
#endif
        /* The batch's leading run of PLAIN steps is committed at once: a step that interacts,
         * neither stops, roulettes, scatters nor is absorbed changes the state only by w *= fac,
         * tau += d_tau, one draw and the coefficients it leaves -- every lane decides its step from
         * the weight before it (the sequential product, in the serial order, so bit-identical) and
         * the draw at its counter; the first lane that is not plain ends the run, and its step (and
         * the rest of the batch) goes through the serial code below. */
        int bj0 = 0;
        {
            /* weight and optical depths before step j (lane j), and after all nb steps (lane nb) */
            double w_run = w, ta_run = tau_abs, ts_run = tau_scatt;
            double w_j = w, ta_j = tau_abs, ts_j = tau_scatt;
            for (int j = 0; j < nb; ++j) {
                if (lane == j) {
                    w_j = w_run;
                    ta_j = ta_run;
                    ts_j = ts_run;
                }
                w_run = w_run * bcast(l_fac, j);
                ta_run = ta_run + bcast(l_dta, j);
                ts_run = ts_run + bcast(l_dts, j);
            }
            if (lane == nb) {
                w_j = w_run;
                ta_j = ta_run;
                ts_j = ts_run;
            }
            /* the window of draws must hold counters rng.ctr .. rng.ctr + nb - 1 */
            if (rng.ctr - wbase + (uint32_t)nb > 64u) {
                wbase = rng.ctr;
                Rng g = rng;
                g.ctr = wbase + (uint32_t)lane;
                win = uniform(g);
            }
            const double u = __shfl(win, (int)(rng.ctr - wbase) + (lane < nb ? lane : 0));
            /* the state before step j: lane j - 1's results, or the carried ones for j = 0 */
            const double up_x1 = __shfl_up(l_x1, 1), up_ne = __shfl_up(l_ne, 1);
            const double up_as = __shfl_up(l_as, 1), up_aa = __shfl_up(l_aa, 1);
            const double x1_prev = lane == 0 ? x1 : up_x1;
            const double ne_prev = lane == 0 ? fl_ne : up_ne, as_prev = lane == 0 ? a_si : up_as,
                         aa_prev = lane == 0 ? a_ai : up_aa;
            /* bias_func with the weight cap (:1391-1404) and the interaction's bias (:977) */
            double bf = 0.0;
            if (!l_zero) {
                const double max = w_j * (0.5 / WEIGHT_MIN);
                double b = l_b0;
                if (b > max) b = max;
                bf = b * (1.0 / TP_OVER_TE);
            }
            const double up_bf = __shfl_up(bf, 1);
            const double bi_prev = lane == 0 ? bi : up_bf;
            const double bias = l_zero ? 0.0 : 0.5 * (bi_prev + bf);
            const double bdt = bias * l_dts;
            const bool may = bdt > (1.0 - u) * (1.0 - 0x1p-40);
            const double lx = may ? -flog(u) : 0.0;
            bool scatter = may && bdt > lx;
            if (scatter) scatter = fdiv(w_j, bias) > WEIGHT_MIN;
            const bool plain = lane < nb && !(x1_prev < P.x1_min) && !(x1_prev > P.x1_max) && !(w_j < WEIGHT_MIN) &&
                               !(l_x1 < P.x1_min) && !(l_x1 > P.x1_max) && !isnan(l_x1) &&
                               (aa_prev > 0.0 || as_prev > 0.0 || ne_prev > 0.0) && !scatter && !(l_dta > 100) &&
                               n_step + lane + 1 <= MAX_N_STEP;
            const unsigned long long np = __ballot(!plain);
            bj0 = np ? __ffsll((long long)np) - 1 : 64; /* lanes >= nb are not plain: bj0 <= nb */
            if (bj0 > 0) {
                const int l = bj0 - 1;
                w = bcast(w_j, bj0);
                tau_abs = bcast(ta_j, bj0);
                tau_scatt = bcast(ts_j, bj0);
                x1 = bcast(l_x1, l);
                fl_ne = bcast(l_ne, l);
                a_si = bcast(l_as, l);
                a_ai = bcast(l_aa, l);
                bi = bcast(bf, l);
                rng.ctr += (uint32_t)bj0;
                n_step += bj0;
                steps += (unsigned long long)bj0;
                since += (unsigned)bj0;
                cur = base + (unsigned long long)l;
                si = base + (unsigned long long)bj0;
                if (own) __hip_atomic_store(&pr.ctl.cons, si, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        for (int bj = bj0; bj < nb; ++bj) {
            ++since;
            /* while (!stop_criterion(photon)) (:919) */
            if (lone_stop(P, x1, w, rng, win, wbase, lane)) {
                ended = done = true;
                break;
            }
            /* photon_2, step size and push of this step: from the geometry wave */
            cur = base + bj;
            x1 = bcast(l_x1, bj);
            ++steps;
            if (lone_stop(P, x1, w, rng, win, wbase, lane)) { /* :932-934 */
                ended = done = true;
                break;
            }
            if (isnan(x1)) { /* a NaN position is absorbing (see transport_trip) */
                if (own) atomicAdd(&C.ctr->n_nan, 1ull);
                ended = done = true;
                reason = 3;
                break;
            }
            if (a_ai > 0.0 || a_si > 0.0 || fl_ne > 0.0) { /* :937 */
                const bool zero = __builtin_amdgcn_readlane(l_zero, bj) != 0;
                fl_ne = bcast(l_ne, bj);
                double d_tau_scatt = bcast(l_dts, bj), d_tau_abs = bcast(l_dta, bj), bf = 0.0, bias = 0.0;
                if (!zero) { /* bias_func's weight cap (:1391-1404) */
                    const double max = w * (0.5 / WEIGHT_MIN);
                    double b = bcast(l_b0, bj);
                    if (b > max) b = max;
                    bf = b * (1.0 / TP_OVER_TE);
                    bias = 0.5 * (bi + bf);
                }
                a_si = bcast(l_as, bj);
                a_ai = bcast(l_aa, bj);
                bi = bf;
                /* x1 = -log u, settled without the logarithm when possible (as in transport_trip) */
                const double u = lone_draw(rng, win, wbase, lane);
                const double bdt = bias * d_tau_scatt;
                const bool may = bdt > (1.0 - u) * (1.0 - 0x1p-40);
                const double lx = may ? -flog(u) : 0.0;
                bool scatter = may && bdt > lx;
                double wc = 0.0;
                if (scatter) { /* w / bias only when it decides (:985) */
                    wc = fdiv(w, bias);
                    scatter = wc > WEIGHT_MIN;
                }
                if (scatter) { /* :985 */
                    const double frac = fdiv(lx, bias * d_tau_scatt);
                    d_tau_abs *= frac;
                    if (d_tau_abs > 100) { /* absorbed before scattering */
                        ended = done = true;
                        reason = 2;
                        break;
                    }
                    d_tau_scatt *= frac;
                    const double d_tau = d_tau_abs + d_tau_scatt;
                    if (d_tau_abs < 1.0e-3)
                        w *= (1.0 - d_tau * (1.0 / 24.0) * (24.0 - d_tau * (12.0 - d_tau * (4.0 - d_tau))));
                    else
                        w *= fexp(-d_tau);
                    /* photon_2 pushed to the scattering point (:1005-1010), by this wave */
                    double x[4], k[4], dk[4], e_0_s;
                    /* photon_2 of this step: the state after the step before, or the restart state */
                    unpack13(base + bj == gen_start ? pr.ctl.rs : pr.ring[(base + bj - 1) % LONE_RING].out, x, k, dk,
                             e_0_s);
                    walk_push(P, x, k, dk, e_0_s, pr.ring[(base + bj) % LONE_RING].dl * frac, 0, 0u, rank, 0);
                    Trig T;
                    Gcov G;
                    ZoneFetch Z;
                    zone_fetch(P, x, Z);
                    trig_at(P, x, T);
                    gcov_from_trig(P, T, G);
                    Fluid F;
                    fluid_from(P, x, G, Z, F);
                    fl_ne = F.n_e;
                    x1 = x[1];
                    cur = LONE_STOP; /* the state is the restart state from here on */
                    if (F.n_e > 0.0 && (k[0] > 1.0e5 || k[0] < 0.0 || isnan(k[0]) || isnan(k[1]) || isnan(k[3]))) {
                        /* scatter_super_photon's parent-side check (:1076-1081, :1018-1021) */
                        k[0] = fabs(k[0]);
                        w = 0.0;
                        if (own) pack13(pr.ctl.rs, x, k, dk, e_0_s);
                        ended = done = true;
                        reason = 2;
                        break;
                    }
                    const double nu2 = fluid_nu(k, F);
                    double a_s2 = 0.0, a_a2 = 0.0;
                    if (!(nu2 < 0.0)) radiation_coeffs(P, k, F, nu2, a_s2, a_a2);
                    const double bf2 = bias_func(bias_d, F.theta_e, w);
                    if (F.n_e > 0.0) {
                        /* the child (:1015-1024): on the early worker into its queue, tracked by the
                         * next free pair; else to the overflow pool, tracked by the relaunch */
                        if (own) {
                            if (kids)
                                queue_child_push(C, kids, x, k, rng, n_scatt, cold, F, wc);
                            else
                                push_overflow(C, x, k, rng, n_scatt, cold, F, wc);
                        }
                        ++children;
                    }
                    a_si = a_s2;
                    a_ai = a_a2;
                    bi = bf2;
                    /* the photon goes on from the scattering point: restart the geometry wave there */
                    ++gen;
                    gen_start = base + bj + 1;
                    if (own) {
                        pack13(pr.ctl.rs, x, k, dk, e_0_s);
                        __hip_atomic_store(&pr.ctl.req, ((unsigned long long)gen << 32) | (base + bj + 1),
                                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    /* the end of the step here, and the end of the batch (the rest of it is on the old
                     * geodesic): the batch's lane values are dead on this path */
                    tau_abs += d_tau_abs;
                    tau_scatt += d_tau_scatt;
                    ++n_step; /* :1058-1063 */
                    if (n_step > MAX_N_STEP) {
                        ended = done = true;
                        reason = 3;
                        break;
                    }
                    si = base + bj + 1;
                    if (own) __hip_atomic_store(&pr.ctl.cons, si, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                } else {
                    if (d_tau_abs > 100) { /* absorbed */
                        ended = done = true;
                        reason = 2;
                        break;
                    }
                    w *= bcast(l_fac, bj);
                }
                tau_abs += d_tau_abs;
                tau_scatt += d_tau_scatt;
            }
            ++n_step; /* :1058-1063 */
            if (n_step > MAX_N_STEP) {
                ended = done = true;
                reason = 3;
                break;
            }
            si = base + bj + 1;
            if (own) __hip_atomic_store(&pr.ctl.cons, si, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#ifdef GRM_TIMING
        ti[3] += __builtin_amdgcn_s_memtime() - tb1;
#endif
    }
#ifdef GRM_TIMING
    /* slots 36-39: photons of > 1e5 steps, 40-43: the others */
    if (own)
        for (int r = 0; r < 4; ++r) atomicAdd(C.timing + (steps > 100000 ? 36 : 40) + r, ti[r]);
#endif
    gen_io = gen;
    if (own) {
        /* the photon's state: the end of step cur (its ring slot is not overwritten before this wave
         * consumes the step after it), or the restart state */
        double x[4], k[4], dk[4], e_0_s;
        unpack13(cur == LONE_STOP ? pr.ctl.rs : pr.ring[cur % LONE_RING].out, x, k, dk, e_0_s);
        if (abandoned) {
            const unsigned long long slot = atomicAdd(C.stuck_count, 1ull);
            if (slot < C.stuck_cap) {
                double *r = C.stuck + slot * STUCK_WORDS;
                r[0] = (double)rng.id;
                r[1] = n_step;
                r[2] = r[3] = r[4] = r[7] = 0.0;
                r[5] = w;
                r[6] = e_0_s;
                for (int i = 0; i < 4; ++i) {
                    r[8 + i] = x[i];
                    r[12 + i] = k[i];
                }
            }
            atomicAdd(&C.ctr->n_abandoned, 1ull);
        } else if (ended) {
            /* record_criterion (:1066) when the stop criterion ended it, else the reason's trace */
            if (reason < 0 && x[1] > P.x1_max && n_step <= MAX_N_STEP)
                record_photon(P, C, cold, rng.id, w, x[1], x[2], x[3], tau_abs, tau_scatt, n_scatt, n_step,
                              reinterpret_cast<double *>(C.spec), (int)(sizeof(grm_spectrum_cell) / sizeof(double)));
            else if (C.trace)
                write_trace(C, cold, rng.id, w, x[1], x[2], x[3], tau_abs, tau_scatt, n_scatt, n_step,
                            reason < 0 ? 2 : reason, -1, -1);
        }
        flush_counters(C);
        atomicAdd(&C.ctr->n_steps, steps);
        if (children) atomicAdd(&C.ctr->n_children, children);
        atomicMax(&C.ctr->max_nstep, (unsigned long long)n_step);
        if (n_step > 100000) atomicAdd(&C.ctr->n_long, 1ull);
    }
}

#ifdef GRM_LONE_TU
__device__ __forceinline__ bool child_setup_body(const Params &P, const Ctl &C, LoneRec *r, int lane);

constexpr unsigned long long LK_STANDBY = 4; /* lone pairs that wait for children once their photon has ended */
#ifndef GRM_LK_SLEEP
#define GRM_LK_SLEEP 32
#endif

/* A lone pair after its own photon (GRM_OPT_EARLY_CHILDREN): the children the kernel's photons append
 * to lk_q, taken in order by whichever pair looks first, for as long as any pair still tracks a
 * photon (*lk_active), so that a long photon's child starts at once instead of in the relaunch after
 * the kernel.  A pair that finds the queue empty waits, up to LK_STANDBY pairs, or leaves.  Leaving
 * is safe whenever the queue is empty: a child is only appended by a pair that is tracking, and
 * every pair looks at the queue again when its photon ends.  Whole wave, uniform control. */
__device__ void lone_children(const Params &P, const Ctl &C, int lane, LonePair &pr, unsigned &gen,
                              unsigned long long n_handed) {
    bool standing = false;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
        /* every handed-over photon finished (its pair may not have started yet when a pair looks) */
        const bool orig_done =
            __hip_atomic_load(C.lk_orig, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= n_handed;
        const unsigned long long act = __hip_atomic_load(C.lk_active, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long taken = __hip_atomic_load(C.lk_taken, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long tail = __hip_atomic_load(C.lk_tail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (tail > C.lk_cap) tail = C.lk_cap;
        if (taken < tail) {
            /* counted as tracking before the claim, so that no waiting pair leaves in between */
            unsigned long long got = ~0ull;
            if (lane == 0) {
                atomicAdd(C.lk_active, 1ull);
                unsigned long long want = taken;
                if (__hip_atomic_compare_exchange_strong(C.lk_taken, &want, taken + 1, __ATOMIC_ACQ_REL,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                    got = taken;
                else
                    atomicAdd(C.lk_active, ~0ull);
            }
            got = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(got >> 32)) << 32) |
                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)got);
            if (got == ~0ull) continue;
            if (standing && lane == 0) atomicAdd(C.lk_standby, ~0ull);
            standing = false;
            while (__hip_atomic_load(C.lk_ready + got, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != C.lk_tag)
                __builtin_amdgcn_s_sleep(1);
            LoneRec *r = C.lk_q + got;
            if (child_setup_body(P, C, r, lane)) lone_interact(P, C, *r, lane, pr, gen, 2);
            if (lane == 0) __hip_atomic_fetch_add(C.lk_active, ~0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        if (act == 0 && orig_done) break; /* nothing queued or tracked, nothing to come: no child can */
        if (!standing) {
            unsigned long long sb = 0;
            if (lane == 0) sb = atomicAdd(C.lk_standby, 1ull);
            sb = (unsigned long long)__builtin_amdgcn_readfirstlane((int)sb);
            if (sb >= LK_STANDBY) {
                if (lane == 0) atomicAdd(C.lk_standby, ~0ull);
                return;
            }
            standing = true;
        }
        /* a guard, not a path: every tracked photon ends within its own watchdog */
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2 * (C.watchdog_ticks ? C.watchdog_ticks : 6000000000ull)) {
            if (lane == 0) __hip_atomic_store(&C.ctr->abort, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(GRM_LK_SLEEP);
    }
    if (standing && lane == 0) atomicAdd(C.lk_standby, ~0ull);
}

/* launched on lone_cap workgroups; the launch before handed over *C.lone_count photons, one to each of
 * the first workgroups; with GRM_OPT_EARLY_CHILDREN the next LK_STANDBY workgroups (as the grid
 * allows) start as standby pairs for the children, so that a launch of few photons -- a relaunch's
 * long photon -- does not track its photons' children one after another on their own pairs */
__global__ __launch_bounds__(128) void lone_kernel(Params P, Ctl C) {
    unsigned long long n_handed = __hip_atomic_load(C.lone_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n_handed > C.lone_cap) n_handed = C.lone_cap;
    const bool extra = blockIdx.x >= n_handed;
    if (blockIdx.x >= C.lone_cap || (extra && (!C.lk_on || n_handed == 0 || blockIdx.x >= n_handed + LK_STANDBY)))
        return;
    const int wave = (int)(threadIdx.x >> 6);
    const int lane = (int)(threadIdx.x & 63);
    LonePair &pr = s_pair[0];
    if (threadIdx.x < 8) s_cnt[threadIdx.x >> 2][threadIdx.x & 3] = 0;
    if (threadIdx.x < LONE_RING) pr.ring[threadIdx.x].tag = 0;
    if (threadIdx.x == 0) {
        pr.ctl.cons = 0;
        pr.ctl.req = 0;
    }
    __syncthreads();
    if (wave == 1) {
        lone_geometry(P, C, lane, pr);
        return;
    }
    unsigned gen = 0;
    if (!extra) {
        if (C.lk_on && lane == 0) atomicAdd(C.lk_active, 1ull);
        lone_interact(P, C, C.lone[blockIdx.x], lane, pr, gen, C.lk_on ? 2 : 0);
        if (C.lk_on && lane == 0) {
            /* its children are queued before it counts as finished (release) */
            __hip_atomic_fetch_add(C.lk_orig, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(C.lk_active, ~0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (C.lk_on) lone_children(P, C, lane, pr, gen, n_handed);
    if (lane == 0) __hip_atomic_store(&pr.ctl.req, LONE_STOP, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* Concurrent worker for long photons (one workgroup of LONE_PAIRS two-wave pairs on a second
 * stream, beside the bulk launch): once it runs (early_live), a lane-loop photon that reaches early_steps steps is
 * handed over at the top of a step into the early queue (slot claimed by early_tail, published by
 * early_ready[slot] = early_tag); each pair's interaction wave claims slots in order (early_head),
 * waits for them to be published and tracks them with its geometry wave.  It exits once the bulk
 * launch has ended (early_done, set by its last workgroup) and every claimed slot is done.  Without
 * it such a photon would advance one step per lane-loop trip (~7 us) until the bulk ends. */
/* A child request in a queue slot r (queue_child_push) made a photon at the top of its first
 * step: scatter_super_photon's sampling and the set-up at the head of track_super_photon
 * (harm_model.cpp:1083-1215, 895-917) -- the lane loop's sample_child, init_photon and set-up trip,
 * with the same functions: dk/dlambda from the connection at x (its zero-length push), the fluid,
 * both coefficients and the bias at x -- written back into the slot as the LoneRec a hand-over would
 * be.  The whole wave, identical values in every lane; lane 0 writes.  false = an invalid child
 * (traced with reason 4, as in the lane loop). */
/* Inlined.  Out of line (a call) the early kernel's serial chain ran 1.299-1.307 us/step against
 * 1.306-1.313 inlined (tools/gpu_kids_ab.sh), but the same call from lone_kernel handed lone_interact
 * records whose weight came out NaN (every child of the lone kernel's photons; profiles/
 * r06_early_children/lk_debug.log) while the inlined body is photon-by-photon exact in both kernels. */
__device__ __forceinline__ bool child_setup_body(const Params &P, const Ctl &C, LoneRec *r, int lane) {
    SReq R;
    load_sreq(reinterpret_cast<const SReq *>(r), R);
    Rng rng;
    rng.k0 = C.key0;
    rng.k1 = C.key1;
    double x[4], k[4], w;
    Cold c;
    if (lane == 0) atomicAdd(&C.ctr->n_tracked, 1ull);
    bool ok = sample_child_core(P, R, rng, x, k, w, &c);
    ok = ok && !(isnan(x[0]) || isnan(x[1]) || isnan(x[2]) || isnan(x[3]) || isnan(k[0]) || isnan(k[1]) ||
                 isnan(k[2]) || isnan(k[3]) || w == 0.0);
    if (!ok) {
        /* both of the lane loop's invalid-child traces carry these values (id, weight, x of the
         * request, no steps) */
        if (lane == 0 && C.trace)
            write_trace(C, &c, R.id, R.w, R.x[1], R.x[2], R.x[3], 0.0, 0.0, R.n_scatt, 0, 4, -1, -1);
        return false;
    }
    Trig T;
    trig_at(P, x, T);
    Gcov G;
    gcov_from_trig(P, T, G);
    double dk[4];
    {
        Conn Cn;
        connection(P, T, Cn);
#pragma unroll
        for (int i = 0; i < 4; ++i) dk[i] = geo_rhs(Cn, i, k);
    }
    ZoneFetch Z;
    zone_fetch(P, x, Z);
    Fluid F;
    fluid_from(P, x, G, Z, F);
    const double nu = fluid_nu(k, F);
    double a_s = 0.0, a_a = 0.0;
    radiation_coeffs(P, k, F, nu, a_s, a_a); /* the set-up evaluates them whatever nu (transport_trip) */
    const double bf = bias_func(bias_den(P, C), F.theta_e, w);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            r->x[i] = x[i];
            r->k[i] = k[i];
            r->dk[i] = dk[i];
        }
        r->w = w;
        r->e_0_s = c.e;
        r->tau_abs = 0.0;
        r->tau_scatt = 0.0;
        r->a_si = a_s;
        r->a_ai = a_a;
        r->bi = bf;
        r->fl_ne = F.n_e;
        r->c = c;
        r->id = rng.id;
        r->ctr = rng.ctr;
        r->n_step = 0;
        r->n_scatt = R.n_scatt;
        r->pad = 0;
    }
    __threadfence(); /* the wave reads the record back (lone_interact) */
    return true;
}

/* the early worker's next queue slot for the calling interaction wave, or ~0 when none will come.
 * Out of line (it touches only global memory): the kernel's SGPR spills 344 -> 265 */
__device__ __attribute__((noinline)) unsigned long long early_claim(const Ctl &C, unsigned long long rt_start) {
    unsigned long long slot = 0;
    if ((threadIdx.x & 63) == 0) slot = atomicAdd(C.early_head, 1ull);
    slot = (unsigned long long)__builtin_amdgcn_readfirstlane((int)slot); /* < 2^31 */
    unsigned long long t_done = 0; /* when this wave first saw the bulk launch ended */
    while (true) {
        if (slot < C.early_cap &&
            __hip_atomic_load(C.early_ready + slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == C.early_tag)
            return slot;
        if (__hip_atomic_load(C.early_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            /* the bulk launch has ended: every claimed hand-over is published, so a slot past the
             * claims (or past the queue) will never come -- unless a pair still tracking a photon may
             * append a child (queue_child_push).  Slots finish in any order, but while this slot is
             * unpublished every later one is too, so *early_fin >= slot says that every slot before
             * it is finished: nothing is left that could append.  *early_fin is read before the tail
             * (a pair appends before it counts its slot finished), and a pair that leaves counts its
             * own slot, so the pair holding the next one can leave in turn. */
            if (slot >= C.early_cap) return ~0ull;
            const unsigned long long fin =
                C.early_kids_on ? __hip_atomic_load(C.early_fin, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) : 0;
            const unsigned long long tail = __hip_atomic_load(C.early_tail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (slot >= tail && (!C.early_kids_on || fin >= slot)) {
                if (C.early_kids_on && (threadIdx.x & 63) == 0)
                    __hip_atomic_fetch_add(C.early_fin, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                return ~0ull;
            }
            /* a guard, not a path: the other pair's photon ends within its own watchdog; a count
             * that never arrives (a bug) fails the call instead of keeping the GPU */
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (t_done == 0) t_done = now;
            if (now - t_done > 2 * (C.watchdog_ticks ? C.watchdog_ticks : 6000000000ull)) {
                if ((threadIdx.x & 63) == 0) __hip_atomic_store(&C.ctr->abort, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return ~0ull;
            }
        }
        if (__builtin_amdgcn_s_memrealtime() - rt_start > EARLY_ALONE_TICKS &&
            __builtin_amdgcn_readfirstlane(
                (int)__hip_atomic_load(C.bulk_live, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
            /* no bulk workgroup has started: the launches are serialised and this one runs first.
             * Close the queue, then leave unless a bulk workgroup started meanwhile (then reopen
             * it: a workgroup that read 1 after starting is seen here by the store-load order) */
            if ((threadIdx.x & 63) == 0) __hip_atomic_store(C.early_live, 2ull, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane(
                    (int)__hip_atomic_load(C.bulk_live, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT)) == 0)
                return ~0ull;
            if ((threadIdx.x & 63) == 0) __hip_atomic_store(C.early_live, 1ull, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
        }
        __builtin_amdgcn_s_sleep(64);
    }
}

__global__ __launch_bounds__(64 * 2 * LONE_PAIRS) void early_kernel(Params P, Ctl C) {
    const int wave = (int)(threadIdx.x >> 6);
    const int lane = (int)(threadIdx.x & 63);
    LonePair &pr = s_pair[wave >> 1];
    if (threadIdx.x < 4 * 2 * LONE_PAIRS) s_cnt[threadIdx.x >> 2][threadIdx.x & 3] = 0;
    if (lane < LONE_RING) pr.ring[lane].tag = 0;
    if (lane == 0) {
        pr.ctl.cons = 0;
        pr.ctl.req = 0;
    }
    __syncthreads();
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) __hip_atomic_store(C.early_live, 1ull, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
    if (wave & 1) {
        /* one inlined copy per pair: the pair's LDS block at a constant address, as in lone_kernel
         * (with the block indexed by the wave the geometry step compiled to ~20 more instructions and
         * ran 1.39 us per step against the lone kernel's 1.29-1.31; now 1.32-1.37) */
        if (wave == 1)
            lone_geometry(P, C, lane, s_pair[0]);
        else
            lone_geometry(P, C, lane, s_pair[1]);
        return;
    }
    unsigned gen = 0;
    while (true) {
        const unsigned long long slot = early_claim(C, rt_start);
        if (slot == ~0ull) break;
        LoneRec *r = C.early_q + slot;
        /* a child request (pad = 1, wave-uniform) becomes a photon at the top of its first step */
        const bool go = r->pad != 1 || child_setup_body(P, C, r, lane);
        if (go) lone_interact(P, C, *r, lane, pr, gen, C.early_kids_on ? 1 : 0);
        if (C.early_kids_on && lane == 0)
            __hip_atomic_fetch_add(C.early_fin, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) __hip_atomic_store(&pr.ctl.req, LONE_STOP, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

#endif /* GRM_LONE_TU */

#if !defined(GRM_LONE_TU) && !defined(GRM_SPLIT_TU)
/* One trip of the lane state machine = at most ONE geodesic push attempt, then, if that attempt
 * completed a step, the rest of the while-loop body of track_super_photon
 * (harm_model.cpp:919-1063).  A lane that has to halve its step (push_photon's recursion,
 * :1279-1285) spends extra trips while the other lanes of the wave keep stepping, instead of the
 * whole wave waiting for the deepest halving tree.  `walked`: halving_walk has just completed this
 * lane's push (its phase-0 block ran before it).  Returns false when the photon's life ended. */
__device__ bool transport_trip(const Params &P, const Ctl &C, Lane &L, Cold *cold, SReq *wstack, int *wtop,
                               const Slot &ph2, const Slot &bk, double bias_d, bool walked, bool &stepped) {
    if (L.phase == 0 && !trip_begin(P, C, L, cold, ph2)) return false;
    TSTAMP(8);
    /* one attempt of push_photon at the current node of the halving tree (:1217-1289).  A lane in
     * set-up (phase 3) makes a zero-length attempt instead: x and k stay, the corrector's first pass
     * leaves dk = dk/dlambda from the connection at x -- init_dkdlam (:915, :1571-1587) -- and T, G
     * are then at x for the fluid evaluation below. */
    const bool setup = L.phase == 3;
    Trig T;
    Gcov G;
    ZoneFetch Z;
    bool have_tg = false;
    TLANES(18, !walked && (setup || !(L.x[1] < P.xs1))); /* slots 18-19: push attempts */
    if (!walked && (setup || !(L.x[1] < P.xs1))) {
        if (L.depth > 0) {
            save_xkdk(bk, L);
        }
        double e_1;
        const bool fail = push_attempt(P, L.x, L.k, L.dk, L.e_0_s, ldexp(L.hlen, -L.depth), e_1, T, G);
        TSTAMP(9);
        if (setup) {
            /* restore x, k exactly (a non-finite dk must not leak into them through 0 * dk) */
#pragma unroll
            for (int i = 0; i < 3; ++i) L.x[1 + i] = ph2[i];
#pragma unroll
            for (int i = 0; i < 4; ++i) L.k[i] = ph2[3 + i];
        } else if (fail && L.depth < MAX_SUBDIV) {
            if (L.depth == 0) {
                load_ph2(ph2, L);
            } else {
                load_xkdk(bk, L);
            }
            ++L.depth;
            L.pend |= 1u << L.depth;
            return true;
        }
        if (!setup) L.e_0_s = e_1;
        have_tg = true;
    }
    if (L.pend) {
        L.depth = 31 - __builtin_clz(L.pend);
        L.pend &= ~(1u << L.depth);
        return true;
    }
    /* the push is complete.  Phase 1 = end of a geodesic step: stop test, then the interaction
     * block (:927-1056).  Phase 2 = back at the scattering point after the re-push (:1005-1055).
     * Both evaluate the fluid and the absorption/scattering coefficients at the new point; they share
     * ONE evaluation here so a wave with lanes in both phases runs that code once. */
    const bool at_scatter = L.phase == 2;
    if (!at_scatter && !setup) {
        stepped = true; /* counted per wave by the caller (a ballot), not per lane in LDS */
        if (stop_criterion(P, L)) {
            end_of_life(P, C, cold, L);
            return false;
        }
        /* A NaN position is absorbing: every later stop test is false, no interaction can fire
         * (bias * d_tau_scatt > x1 is false for NaN), and record_super_photon drops NaN photons
         * (harm_model.cpp:1291-1295), so the reference's loop only burns steps -- each a full
         * 255-attempt halving tree, since err is NaN -- until max_n_step (:1058-1063, no record :1066).  End it here
         * with the same (empty) outcome. */
        if (isnan(L.x[1])) {
            atomicAdd(&C.ctr->n_nan, 1ull);
            trace_end(C, cold, L, 3);
            return false;
        }
    }
    TSTAMP(10);
    TLANES(16, setup || at_scatter || L.alpha_absi() > 0.0 || L.alpha_scatti() > 0.0 || L.fl_ne() > 0.0);
    if (setup || at_scatter || L.alpha_absi() > 0.0 || L.alpha_scatti() > 0.0 || L.fl_ne() > 0.0) {
        if (!have_tg) {
            trig_at(P, L.x, T);
            gcov_from_trig(P, T, G);
        }
        zone_fetch(P, L.x, Z);
        Fluid F;
        fluid_from(P, L.x, G, Z, F);
        L.fl_ne() = F.n_e;
        TSTAMP(11);
        /* scatter_super_photon's parent-side check (:1076-1081) */
        if (at_scatter && F.n_e > 0.0 &&
            (L.k[0] > 1.0e5 || L.k[0] < 0.0 || isnan(L.k[0]) || isnan(L.k[1]) || isnan(L.k[3]))) {
            L.k[0] = fabs(L.k[0]);
            L.w = 0.0;
            trace_end(C, cold, L, 2);
            return false;
        }
        /* phase 1 skips the coefficients out of the fluid (bound_flag, :941-955); both skip them
         * for nu < 0 */
        const double nu = fluid_nu(L.k, F);
        const bool zero = !setup && (nu < 0.0 || (!at_scatter && F.n_e == 0.0));
        double a_s = 0.0, a_a = 0.0;
        if (!zero) {
            radiation_coeffs(P, L.k, F, nu, a_s, a_a);
        }
        const double bf = (zero && !at_scatter) ? 0.0 : bias_func(bias_d, F.theta_e, L.w);
        TSTAMP(12);
        if (setup) { /* the set-up's coefficients (:905-913); the loop starts on the next trip */
            L.alpha_scatti() = a_s;
            L.alpha_absi() = a_a;
            L.bi() = bf;
            L.phase = 0;
            return true;
        }
        if (at_scatter) {
            /* the child leaves as a scatter request; its stores go out after this trip's table
             * loads, so no load of the trip waits behind them (vmcnt is in order) */
            if (F.n_e > 0.0) {
                if (push_request(C, L.x, L.k, L.rng, L.n_scatt(), cold, F, L.p_wc(), wstack, wtop)) ++L.flight();
                ++L.c_children();
            }
            L.alpha_scatti() = a_s;
            L.alpha_absi() = a_a;
            L.bi() = bf;
            L.tau_abs() += L.p_dtau_abs();
            L.tau_scatt() += L.p_dtau_scatt();
        } else {
            /* trapezoid optical depths over the step (:957-975) */
            const double dl = L.dl;
            double d_tau_scatt, d_tau_abs, bias;
            if (zero) {
                d_tau_scatt = 0.5 * L.alpha_scatti() * P.d_tau_k * dl;
                d_tau_abs = 0.5 * L.alpha_absi() * P.d_tau_k * dl;
                bias = 0.0;
            } else {
                d_tau_scatt = 0.5 * (L.alpha_scatti() + a_s) * P.d_tau_k * dl;
                d_tau_abs = 0.5 * (L.alpha_absi() + a_a) * P.d_tau_k * dl;
                bias = 0.5 * (L.bi() + bf);
            }
            L.alpha_scatti() = a_s;
            L.alpha_absi() = a_a;
            L.bi() = bf;
            /* x1 = -log u (:983); the test bias * d_tau_scatt > x1 is settled without the logarithm
             * when bias * d_tau_scatt <= (1 - u)(1 - 2^-40) <= -log u (margin for the log's rounding) */
            const double u = uniform(L.rng);
            const double bdt = bias * d_tau_scatt;
            const bool may = bdt > (1.0 - u) * (1.0 - 0x1p-40);
            const double x1 = may ? -flog(u) : 0.0;
            const double wc = fdiv(L.w, bias);
            if (may && bdt > x1 && wc > WEIGHT_MIN) {
                const double frac = fdiv(x1, bias * d_tau_scatt);
                d_tau_abs *= frac;
                if (d_tau_abs > 100) {
                    trace_end(C, cold, L, 2);
                    return false; /* absorbed before scattering */
                }
                d_tau_scatt *= frac;
                const double d_tau = d_tau_abs + d_tau_scatt;
                if (d_tau_abs < 1.0e-3)
                    L.w *= (1.0 - d_tau * (1.0 / 24.0) * (24.0 - d_tau * (12.0 - d_tau * (4.0 - d_tau))));
                else
                    L.w *= fexp(-d_tau);
                /* re-push photon_2 by dl*frac to the scattering point (:1005), on later trips */
                load_ph2(ph2, L);
                L.e_0_s = L.ph2_e0s();
                L.hlen = dl * frac;
                L.depth = 0;
                L.pend = 0;
                L.phase = 2;
                L.p_dtau_abs() = d_tau_abs;
                L.p_dtau_scatt() = d_tau_scatt;
                L.p_wc() = wc;
                return true;
            }
            if (d_tau_abs > 100) {
                trace_end(C, cold, L, 2);
                return false; /* absorbed */
            }
            const double d_tau = d_tau_abs + d_tau_scatt;
            if (d_tau < 1.0e-3)
                L.w *= (1.0 - d_tau * (1.0 / 24.0) * (24.0 - d_tau * (12.0 - d_tau * (4.0 - d_tau))));
            else
                L.w *= fexp(-d_tau);
            L.tau_abs() += d_tau_abs;
            L.tau_scatt() += d_tau_scatt;
        }
    }
    TSTAMP(13);
    L.phase = 0;
    ++L.n_step;
    if (L.n_step > MAX_N_STEP) {
        trace_end(C, cold, L, 3);
        return false;
    }
    return true;
}

/* watchdog record of a photon abandoned mid-flight: id, n_step, phase, depth, pend, w, e_0_s, dl, x, k */
__device__ void record_stuck(const Ctl &C, const Lane &L) {
    const unsigned long long slot = atomicAdd(C.stuck_count, 1ull);
    if (slot >= C.stuck_cap) return;
    double *r = C.stuck + slot * STUCK_WORDS;
    r[0] = (double)L.rng.id;
    r[1] = L.n_step;
    r[2] = L.phase;
    r[3] = L.depth;
    r[4] = L.pend;
    r[5] = L.w;
    r[6] = L.e_0_s;
    r[7] = L.dl;
    for (int i = 0; i < 4; ++i) {
        r[8 + i] = L.x[i];
        r[12 + i] = L.k[i];
    }
}

__global__ __launch_bounds__(BLOCK, MIN_WAVES_PER_SIMD) void track_kernel(Params P_, Ctl C_) {
    KArgsK *const ka = kargs();
    const Ctl &C0 = C_;
    const Params &P0 = P_;
#ifdef GRM_TIMING
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) < 24) g_tlds[threadIdx.x >> 6][threadIdx.x & 63] = (threadIdx.x & 63) == 15 ? t_start : 0;
#endif
    __shared__ double lds[2 * LDS_DOUBLES_PER_LANE * BLOCK];
    const Slot ph2{lds + threadIdx.x, BLOCK};
    const Slot bk{lds + LDS_DOUBLES_PER_LANE * BLOCK + threadIdx.x, BLOCK};
    const unsigned lane_id = threadIdx.x & 63;
    const uint64_t gtid = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const int wave = threadIdx.x >> 6;
    SReq *wstack = C0.stack + (gtid >> 6) * WSTACK_CAP;
    __shared__ int s_wtop[BLOCK / 64];
    int *wtop = s_wtop + wave;
    if (lane_id == 0) *wtop = 0;
    if (lane_id == 0) s_recn[wave] = 0;
    if (lane_id < 4) s_cnt[wave][lane_id] = 0;
    if (threadIdx.x == 0 && C0.early_q) __hip_atomic_store(C0.bulk_live, 1ull, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
    /* a multi-rank warm-up: this rank's launch is resident (the job's start barrier) */
    if (threadIdx.x == 0 && C0.n_peers > 1 && C0.admit_n != 0) atomicOr(C0.in_flight, WARM_STARTED);
    __syncthreads();
    Cold *cold = C0.cold + gtid;
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long wave_trips = 0;
    Lane L;
    L.rng.k0 = C0.key0;
    L.rng.k1 = C0.key1;
    bool active = false;
    /* a failed argument check ends the wave at its first trip (the exit path uses C0 only) */
    const bool karg_bad = !kargs_check(ka, P0, C0);
    if (karg_bad && lane_id == 0) atomicAdd(&C0.ctr->karg_bad, 1ull);
    bool pool_done = karg_bad;   /* wave-uniform */
    unsigned long long res_next = 0, res_end = 0; /* wave-uniform: reserved claim positions */
    bool head_done = false;      /* wave-uniform: the pool head has passed pos_end */
    bool warm = !karg_bad && C0.admit_n != 0; /* wave-uniform: warm-up admission in force */
    /* wave-uniform: every rank of the job has started this pass (or the wait gave up); one GPU: true */
    bool started_all = !(C0.n_peers > 1 && C0.admit_n != 0 && C0.start_wait_ticks != 0);
    unsigned wait_trips = 0;     /* consecutive trips idle waiting for admission */
    L.flight() = 0;
    /* wave-uniform; refreshed every trip during the warm-up and every REFRESH_TRIPS trips after it
     * (the device-coherent counters cost a cross-die round trip; past the warm-up they move by
     * parts per million between refreshes) */
    double bias_d = bias_den(P0, C0);
    unsigned trip = 1;
    /* per-lane launch counters, 32-bit in the loop (a lane makes < 2^32 steps per launch), widened
     * for the wave reduction at exit */
    L.c_tracked() = L.c_primaries() = L.c_children() = 0;
    unsigned long long wave_steps = 0; /* wave-uniform: transport steps the wave's lanes completed */
    L.c_nstep_max() = L.c_long() = 0; /* longest photon life; lives > 100k steps */
    const unsigned long long lt_mask = (lane_id == 0) ? 0ull : (~0ull >> (64 - lane_id));

    while (true) {
        KArgsK *const kt = karg_fresh(ka); /* one opaque pointer for both (two would both spill) */
        const Params &P = karg_params(kt);
        const Ctl &C = karg_ctl(kt);
        ++wave_trips;
        TCOUNT(4);
        if (warm && (blockIdx.x >= WARM_BLOCKS || (unsigned)wave >= WARM_WAVES)) {
            /* the warm-up's admission batches are small: the waves of the first WARM_BLOCKS
             * workgroups take them, the rest wait here without touching the counters (their polling
             * would contend with the warm-up's own counter traffic) until the admission is over */
            unsigned long long end = 0;
            if (lane_id == 0) end = __hip_atomic_load(C.admit_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane((int)(end >> 32)) != -1 ||
                __builtin_amdgcn_readfirstlane((int)end) != -1) {
#pragma unroll
                for (int z = 0; z < GRM_PARK_SLEEPS; ++z) __builtin_amdgcn_s_sleep(127);
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
                if (stop) { /* abandon: drop the lane photons, the wave's stack and the pool; exit */
                    /* end the admission too, so that waves parked for it wake up and exit */
                    if (lane_id == 0) __hip_atomic_store(C.admit_end, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (lane_id == 0 && C.n_peers > 1) atomicOr(C.in_flight, WARM_DONE);
                    if (active) {
                        record_stuck(C, L);
                        atomicAdd(&C.ctr->n_abandoned, 1ull);
                        active = false;
                    }
                    pool_done = true;
                    warm = false;
                    if (lane_id == 0) *wtop = 0;
                }
            }
            TSTAMP(7);
        }
        if (__builtin_amdgcn_readfirstlane(s_recn[wave]) >= RECBUF_FLUSH) flush_records(C);
        /* Refill (converged point).  A primary needs only its loads here (its set-up runs in the
         * trip, phase 3), so idle lanes take primaries as soon as refill_min of them are idle.  A
         * child needs the divergent scattering sampling (sample_child), so children go in batches:
         * once child_min wait on the wave's stack, the wave stops taking primaries until as many
         * lanes are idle and samples them together (stack order: depth-first, like the reference's
         * recursion, harm_model.cpp:1023).  With no lane active, or once the pool is drained, the
         * wave refills whatever it can. */
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
                        /* warm-up: claim only inside the admitted batch (CAS); once it is claimed and
                         * nothing is in flight, one wave admits the next batch.  In a multi-rank job
                         * the gate is the job's: every rank's flight against every rank's admitted
                         * photons (warm_job), so the ranks' batches interleave as one GPU's would
                         * (each rank gating on its own flight let the job run ahead of its history:
                         * +5 % recorded at 8 ranks) */
                        long long got = 0;
                        int off = 0;
                        const bool job = C.n_peers > 1;
                        unsigned long long j_hist = 0;
                        long long j_flight = 0;
                        if (job) warm_job(C, j_hist, j_flight);
                        if (!started_all)
                            started_all = job_started(C) || __builtin_amdgcn_s_memrealtime() - rt_start > C.start_wait_ticks;
                        const unsigned long long unit = job ? WARM_HIST + 1 : 1; /* admitted + in flight */
                        if (lane_id == 0) {
                            const unsigned long long end =
                                __hip_atomic_load(C.admit_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (end == ~0ull) {
                                off = 1;
                            } else if (!started_all) {
                                /* the job's start barrier: no claim until every rank's launch runs */
                            } else {
                                const unsigned long long head =
                                    __hip_atomic_load(C.pool_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                base = head;
                                if (head < end) {
                                    unsigned long long want = min((unsigned long long)k_pool, end - head);
                                    if (C.admit_spread) want = min(want, C.admit_spread);
                                    atomicAdd(C.in_flight, want * unit); /* before the claim is visible */
                                    if (atomicCAS(C.pool_head, head, head + want) == head)
                                        got = (long long)want;
                                    else
                                        atomicAdd(C.in_flight, (unsigned long long)(-(long long)(want * unit)));
                                } else if (job ? (unsigned long long)j_flight <= (j_hist >> C.admit_slack)
                                               : __hip_atomic_load(C.in_flight, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <=
                                                     ((C.admit_h0 + end) >> C.admit_slack)) {
                                    /* the next batch once all but a straggler fraction of the history
                                     * has ended: the counters then hold nearly all of it, and one
                                     * long-lived photon does not hold the warm-up up */
                                    /* one GPU: the batch doubles the history, up to admit_lim.  A job
                                     * (n_peers ranks): this rank's share of a batch that doubles the JOB's
                                     * admitted photons, and the admission ends for every rank when the job's
                                     * reach admit_lim (= n_peers x one GPU's); sized from its own history, a
                                     * rank that won a few gate openings ran its batches ahead of the others
                                     * and left the warm-up early, on a history far shorter than the job's
                                     * in flight (+4-5 % recorded at 2-8 emulated ranks, round 4) */
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
                                        /* the admission log: [3 + 2k] when batch k + 1 opened, [4 + 2k]
                                         * the photons then in flight */
                                        const unsigned long long k = atomicAdd(C.phases + 2, 1ull);
                                        if (k < (PHASE_LOG - 3) / 2) {
                                            C.phases[3 + 2 * k] = t;
                                            /* photons in flight: a multi-rank pass block packs them into
                                             * the signed low word of its warm-up state (see DevCounters) */
                                            const unsigned long long f =
                                                __hip_atomic_load(C.in_flight, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                            const long long fl = job ? (long long)(int)(unsigned)f : (long long)f;
                                            C.phases[4 + 2 * k] = (unsigned long long)(fl < 0 ? 0 : fl);
                                        }
                                    }
                                }
                            }
                        }
                        if (__shfl(off, 0)) {
                            warm = false; /* admission over: plain claims from here on */
                        } else {
                            base = __shfl(base, 0);
                            k_pool = (int)__shfl(got, 0);
                            if (k_pool > 0 && base + k_pool >= C.pos_end) pool_done = true;
                        }
                    }
                    if (!warm) {
                        /* the wave's reservation of claim positions: one global atomic per RES_CHUNK
                         * positions instead of one per refill (2048 waves refilling a few lanes every
                         * ~20 trips would queue on the pool head's single address) */
                        if (res_next >= res_end) {
                            unsigned long long b = 0;
                            if (lane_id == 0) b = atomicAdd(C.pool_head, (unsigned long long)RES_CHUNK);
                            b = __shfl(b, 0);
                            res_next = b;
                            res_end = min(b + RES_CHUNK, C.pos_end);
                            head_done = b + RES_CHUNK >= C.pos_end;
                            if (C.phases && lane_id == 0 && b < C.pos_end && head_done)
                                C.phases[1] = __builtin_amdgcn_s_memrealtime(); /* the one wave of the last chunk */
                        }
                        base = res_next;
                        k_pool = res_end > res_next ? (int)min((unsigned long long)k_pool, res_end - res_next) : 0;
                        res_next += k_pool;
                        if (head_done && res_next >= res_end) pool_done = true;
                    }
                }
                if (lane_id == 0) *wtop = top - k_child;
#ifdef GRM_TIMING
                if (k_child) TCOUNT(5);
                if (k_pool) TCOUNT(6);
#endif
                TSTAMP(14);
                bool has = false, ok = true;
                if (!active && r < k_child) {
                    SReq R;
                    load_sreq(wstack + (top - 1 - r), R);
                    ok = sample_child(P, C, R, L, cold);
                    if (!ok && C.trace)
                        write_trace(C, cold, R.id, R.w, R.x[1], R.x[2], R.x[3], 0.0, 0.0, R.n_scatt, 0, 4, -1, -1);
                    has = true;
                }
                TSTAMP(0);
                if (!active && r >= k_child && r - k_child < k_pool) {
                    const unsigned long long pos = base + (unsigned long long)(r - k_child);
                    const unsigned long long idx =
                        (pos & ((1ull << C.pool_sh) - 1)) * C.pool_m + (pos >> C.pool_sh);
                    if (pos < C.pos_end && idx >= C.n_pool) --L.flight(); /* a hole: claimed, ends at once */
                    if (pos < C.pos_end && idx < C.n_pool) {
                        if (C.pool_kind == 0) {
                            load_primary(C, idx, L, cold);
                            ++L.c_primaries();
                        } else {
                            SReq R;
                            load_sreq(reinterpret_cast<const SReq *>(C.pool) + idx, R);
                            ok = sample_child(P, C, R, L, cold);
                            if (!ok && C.trace)
                                write_trace(C, cold, R.id, R.w, R.x[1], R.x[2], R.x[3], 0.0, 0.0, R.n_scatt, 0, 4,
                                            -1, -1);
                        }
                        has = true;
                    }
                }
                if (has) {
                    ++L.c_tracked();
                    if (ok) active = init_photon(C, cold, L, ph2);
                    if (!active) --L.flight(); /* started and ended at once (invalid) */
                }
                TSTAMP(1);
            }
        }
        if (!__any(active)) {
            if (warm) {
                int d = L.flight(); /* flush before waiting: the barrier needs everyone's ends */
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
                if (lane_id == 0 && d) atomicAdd(C.in_flight, (unsigned long long)(long long)d);
                L.flight() = 0;
            }
            if (pool_done && *wtop == 0) break;
            if (warm) {
                /* waiting for the next batch; a barrier that never opens (it cannot, short of a
                 * counting bug) must not hang the GPU: after ~1 s give the warm-up up for all */
                if (++wait_trips > (1u << 21) && lane_id == 0) {
                    __hip_atomic_store(C.admit_end, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (C.n_peers > 1) atomicOr(C.in_flight, WARM_DONE);
                }
                __builtin_amdgcn_s_sleep(16);
            }
            continue;
        }
        wait_trips = 0;
        /* a photon that has run early_steps steps goes to the concurrent early_kernel at the top of
         * a step (one lane-loop trip is ~7 us per step for it, the pair ~1.8 us) */
        if (C.early_q && !warm) {
            const bool early = active && L.phase == 0 && L.n_step >= C.early_steps;
            /* a full queue is read, not claimed: past early_cap every such lane would add to the one
             * tail word on every trip for the rest of the launch */
            if (__ballot(early) && __hip_atomic_load(C.early_live, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT) == 1 &&
                __hip_atomic_load(C.early_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < C.early_cap && early) {
                const unsigned long long slot = atomicAdd(C.early_tail, 1ull);
                if (slot < C.early_cap) {
                    export_lone(C.early_q + slot, L, cold);
                    __threadfence();
                    __hip_atomic_store(C.early_ready + slot, C.early_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    active = false;
                }
            }
        }
        /* the tail: this wave's only work left is one photon -- hand it to the lone-photon kernel at
         * the top of a step (in the test mode GRM_OPT_LONE = 2: every photon at the top of its
         * first step); halving_walk finishes a push already in progress with the whole wave */
        bool walked = false, ended = false;
        const bool tail = pool_done && !warm;
        if (tail || C.lone_all) {
            const unsigned long long act = __ballot(active);
            const int n_act = __popcll(act);
            const bool alone = n_act == 1 && *wtop == 0;
            if (C.lone && (alone || C.lone_all)) {
                /* a full hand-over queue is read, not claimed, and the photons stay in the lane loop
                 * (claiming past the cap and skipping the trip would retry forever) */
                const bool hand = active && L.phase == 0 &&
                                  __hip_atomic_load(C.lone_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < C.lone_cap;
                if (__ballot(hand)) {
                    unsigned long long slot = ~0ull;
                    if (hand) slot = atomicAdd(C.lone_count, 1ull);
                    const bool handed = hand && slot < C.lone_cap;
                    if (handed) {
                        export_lone(C.lone + slot, L, cold);
                        active = false;
                    }
                    if (__ballot(handed)) continue; /* the rest reach the top of a step on later trips */
                }
            }
            if (tail && alone) {
                const int owner = __ffsll((long long)act) - 1;
                int walk = 0;
                if (active) {
                    if (L.phase == 0 && !trip_begin(P, C, L, cold, ph2))
                        ended = true;
                    else
                        walk = (L.phase == 1 || L.phase == 2) ? 1 : 0;
                }
                if (__builtin_amdgcn_readlane(walk, owner)) {
                    halving_walk(P, L, owner);
                    walked = true;
                }
            }
        }
        bool stepped = false;
        if (active) {
            active = !ended && transport_trip(P, C, L, cold, wstack, wtop, ph2, bk, bias_d, walked, stepped);
            if (!active) {
                L.c_nstep_max() = max((int)L.c_nstep_max(), L.n_step);
                L.c_long() += L.n_step > 100000 ? 1 : 0;
                --L.flight();
            }
        }
        wave_steps += (unsigned long long)__popcll(__ballot(stepped)); /* scalar: no LDS round trip per step */
        if (warm) {
            int d = L.flight();
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
            if (lane_id == 0 && d) atomicAdd(C.in_flight, (unsigned long long)(long long)d);
            L.flight() = 0;
        }
        TSTAMP(2);
    }
#ifdef GRM_TIMING
    if (lane_id == 0) {
        g_tlds[threadIdx.x >> 6][3] = __builtin_amdgcn_s_memtime() - t_start;
        for (int r = 0; r < 15; ++r) atomicAdd(C0.timing + r, g_tlds[threadIdx.x >> 6][r]);
        for (int r = 16; r < 24; ++r) atomicAdd(C0.timing + 16 + r, g_tlds[threadIdx.x >> 6][r]);
    }
#endif
    const Ctl &C = C0;
    /* counters, the buffered records, then the workgroup's spectrum, to the global accumulators */
    flush_counters(C);
    flush_records(C);
    __syncthreads();
    double *slice = spec_slice(C);
    for (int i = threadIdx.x; i < SPEC_LDS; i += BLOCK) {
        /* the slice was accumulated by memory-side atomics; read it there and leave it zero for the
         * next launch (padding fields 12..15 stay zero) */
        if ((i & (SPEC_CELL - 1)) >= SPEC_FIELDS) continue;
        const double v = __hip_atomic_load(slice + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v != 0.0) slice[i] = 0.0;
        if (v != 0.0) unsafeAtomicAdd(reinterpret_cast<double *>(C.spec + i / SPEC_CELL) + (i & (SPEC_CELL - 1)), v);
    }
    /* wave-reduce the lane counters, one atomic per wave */
    unsigned long long w_tracked = (unsigned)L.c_tracked();
    unsigned long long w_primaries = (unsigned)L.c_primaries(), w_children = (unsigned)L.c_children();
    unsigned long long w_long = (unsigned)L.c_long(), w_nstep_max = (unsigned)L.c_nstep_max();
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        w_tracked += __shfl_xor(w_tracked, off);
        w_primaries += __shfl_xor(w_primaries, off);
        w_children += __shfl_xor(w_children, off);
        w_long += __shfl_xor(w_long, off);
        w_nstep_max = max(w_nstep_max, (unsigned long long)__shfl_xor(w_nstep_max, off));
    }
    if (lane_id == 0) {
        atomicAdd(&C.ctr->n_steps, wave_steps);
        atomicAdd(&C.ctr->n_tracked, w_tracked);
        atomicAdd(&C.ctr->n_primaries, w_primaries);
        atomicAdd(&C.ctr->n_children, w_children);
        if (w_long) atomicAdd(&C.ctr->n_long, w_long);
        atomicMax(&C.ctr->max_nstep, w_nstep_max);
        if (C.waves) {
            unsigned long long *wr = C.waves + (gtid >> 6) * 4;
            wr[0] = rt_start;
            wr[1] = __builtin_amdgcn_s_memrealtime();
            wr[2] = wave_trips;
            wr[3] = w_tracked;
        }
    }
    if (C.early_q) { /* the last workgroup out tells early_kernel that no hand-over will follow */
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(C.wg_exit, 1ull) == gridDim.x - 1)
                __hip_atomic_store(C.early_done, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

/* Stream-ordered control of the small device words, so that a pass needs no copy or fill
 * (ROCclr blit) kernels: one workgroup sets the words a launch starts from (and, on a reset, the
 * counters and the whole spectrum, grid-stride), then mirrors the counters and the small words into
 * host-mapped memory, which the host reads after the stream synchronises. */
struct CtlOp {
    DevCounters *ctr;
    unsigned long long *small; /* grm_engine::d_small */
    double *spec;              /* zeroed on a reset (n_spec doubles) */
    size_t n_spec;
    DevCounters *h_ctr;        /* host-mapped mirrors (null: no mirror) */
    unsigned long long *h_small;
    unsigned long long val[16]; /* small[i] = val[i] for the bits of set */
    unsigned set;
    int reset, clear_abort;
    unsigned long long max_tau_init_bits;
    int set_warm;                  /* ctr->warm = warm_val (a multi-rank job's warm-up start) */
    unsigned long long warm_val;
};

/* one pass's results into slot `slot` of the stash (grm_engine_stash): the spectrum, then the
 * counters split by their reduction (sum: recorded, scattered, steps, tracked, children, overflow,
 * dropped, primaries, lives > 1e5; max: max tau_scatt bits, longest life) */
constexpr int STASH_SUMS = 9, STASH_MAXS = 2;
__global__ __launch_bounds__(256) void stash_kernel(const double *spec, const DevCounters *ctr, double *st_spec,
                                                    unsigned long long *st_sum, unsigned long long *st_max, int slot,
                                                    int ncell) {
    double *dst = st_spec + (size_t)slot * ncell;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < ncell; i += gridDim.x * 256) dst[i] = spec[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        unsigned long long *s = st_sum + (size_t)slot * STASH_SUMS, *m = st_max + (size_t)slot * STASH_MAXS;
        s[0] = ctr->n_recorded;
        s[1] = ctr->n_scatt;
        s[2] = ctr->n_steps;
        s[3] = ctr->n_tracked;
        s[4] = ctr->n_children;
        s[5] = ctr->n_overflow;
        s[6] = ctr->n_dropped;
        s[7] = ctr->n_primaries;
        s[8] = ctr->n_long;
        m[0] = ctr->max_tau_bits;
        m[1] = ctr->max_nstep;
    }
}

/* the job's bias counters as bias_den forms them (grm_engine_job_counters; tests of the peer mapping) */
__global__ __launch_bounds__(64) void job_counters_kernel(Params P, Ctl C, double *out) {
    const double den = bias_den(P, C);
    unsigned long long sc = 0, rc = 0, mt = 0;
    const int lane = (int)threadIdx.x;
    if (lane < C.n_peers) {
        const DevCounters *pc = C.peers[lane] + C.ctr_slot;
        sc = __hip_atomic_load(&pc->n_scatt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        rc = __hip_atomic_load(&pc->n_recorded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        mt = __hip_atomic_load(&pc->max_tau_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sc += __shfl_xor(sc, o);
        rc += __shfl_xor(rc, o);
        mt = max(mt, (unsigned long long)__shfl_xor(mt, o));
    }
    if (lane == 0) {
        out[0] = den;
        out[1] = (double)sc;
        out[2] = (double)rc;
        out[3] = __longlong_as_double((long long)mt);
    }
}

__global__ __launch_bounds__(256) void ctl_kernel(CtlOp op) {
    if (op.reset)
        for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < op.n_spec; i += (size_t)gridDim.x * 256)
            op.spec[i] = 0.0;
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    if (op.reset) {
        unsigned long long *c = reinterpret_cast<unsigned long long *>(op.ctr);
        for (int i = 0; i < 16; ++i) c[i] = 0;
        op.ctr->max_tau_bits = op.max_tau_init_bits;
    }
    if (op.clear_abort) op.ctr->abort = 0;
    if (op.set_warm) op.ctr->warm = op.warm_val;
    for (int i = 0; i < 16; ++i)
        if ((op.set >> i) & 1u) op.small[i * SMALL_STRIDE] = op.val[i];
    if (op.h_ctr) {
        const unsigned long long *c = reinterpret_cast<const unsigned long long *>(op.ctr);
        unsigned long long *h = reinterpret_cast<unsigned long long *>(op.h_ctr);
        for (int i = 0; i < 16; ++i) h[i] = c[i];
        for (int i = 0; i < 16; ++i) op.h_small[i] = op.small[i * SMALL_STRIDE];
        __threadfence_system();
    }
}
#endif /* !GRM_LONE_TU && !GRM_SPLIT_TU */

} /* namespace */

#if !defined(GRM_LONE_TU) && !defined(GRM_SPLIT_TU)
/* lone_kernel / early_kernel live in grm_lone.hip (the same source, compiled without
 * -disable-machine-licm, see there); Params and Ctl cross as bytes */
extern "C" hipError_t grm_lone_launch(int which, unsigned grid, hipStream_t s, const void *P, size_t p_size,
                                      const void *C, size_t c_size);
#ifdef GRM_WITH_SPLIT
/* split_kernel lives in grm_split.hip (the bulk transport with geometry and interaction waves): an
 * experiment that lost, built only into variant libraries (tools/build_variant.sh) */
extern "C" hipError_t grm_split_launch(unsigned grid, hipStream_t s, const void *P, size_t p_size, const void *C,
                                       size_t c_size);
#endif

/* ========================================================================= */
/* engine object + C ABI                                                      */
/* ========================================================================= */
struct grm_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
    Params P{};
    double *d_zones = nullptr, *d_hot = nullptr, *d_k2 = nullptr;
    DevCounters *d_ctr = nullptr;       /* the counter block in use: d_ctr_own, or a pass slot */
    DevCounters *d_ctr_own = nullptr;   /* allocated with the engine */
    DevCounters *d_ctr_slots = nullptr; /* per-pass blocks (grm_engine_stash_reserve), shared with peers */
    int n_ctr_slots = 0, ctr_slot = -1;
    const DevCounters **d_peers = nullptr; /* device array: every rank's d_ctr_slots */
    int n_peers = 0;
    std::vector<void *> ipc_open;           /* peers' blocks opened by IPC (closed at destroy) */
    grm_spectrum_cell *d_spec = nullptr;
    SReq *d_stack = nullptr;
    Cold *d_cold = nullptr;
    size_t lanes = 0;
    int grid = 0;
    SReq *d_ovf[2] = {nullptr, nullptr};
    unsigned long long ovf_cap = 0;
    unsigned long long *d_small = nullptr; /* [0] pool head, [1..2] ovf counts, [3] trace count,
                                              [4] warm-up in flight, [5] warm-up admitted end */
    grm_init_photon *d_batch = nullptr;
    size_t batch_cap = 0;
    grm_trace *d_trace = nullptr;
    unsigned long long trace_cap = 0;
    uint64_t seed = 123;
    int bias_mode = 0;
    uint64_t id_base = 0;
    int grid_override = 0;
    int64_t flight_ratio = 96; /* GRM_OPT_FLIGHT_RATIO: a live-bias call of n photons runs on <= n / this lanes */
    int split = 0;             /* GRM_OPT_SPLIT: the bulk launch is split_kernel (grm_split.hip) */
    int split_thr = 48, split_spin = 4, split_gthr = 24; /* GRM_OPT_SPLIT_THR / _SPIN / _GTHR (profiles/r05_split) */
    int split_batch = 1; /* GRM_OPT_SPLIT_BATCH */
    double max_tau_init = 0.0;
    bool frozen_set = false;
    /* photons; -1 = lanes; -2 (default) = auto: lanes for a call of fewer than WARMUP_AUTO_RATIO x lanes
     * photons, else WARMUP_PHOTONS (profiles/r03d_warmup_rank_sweep_1e5.log) */
    int64_t warmup = -2;
    int warmup_slack = -1; /* log2; -1 (default) = auto: 4 when the warm-up ramps to a grid of lanes, else 1 */
    int refill_min = 2;      /* primaries: set-up is in the trip (phase 3), so refill early */
    int child_min = 8;       /* children: batch the divergent scattering sampling */
    uint64_t history = 0;    /* primaries tracked since reset */
    double fz_scatt = 0.0, fz_rec = 0.0, fz_maxtau = 0.0;
    grm_stats stats{};
    grm_init_photon *d_upload = nullptr;
    size_t upload_cap = 0;
    ncclComm_t comm = nullptr;
    /* deferred reduction of a job's passes (grm_engine_stash*): per slot the spectrum, 9 summed
     * counters and 2 max counters */
    double *d_stash_spec = nullptr;
    unsigned long long *d_stash_sum = nullptr, *d_stash_max = nullptr;
    int stash_cap = 0;
    unsigned long long *d_timing = nullptr;
    unsigned long long *d_waves = nullptr; /* [lanes / 64][4] per-wave record of the last launch */
    int64_t watchdog_ms = 60000;           /* per-launch watchdog (GRM_OPT_WATCHDOG_MS; 0 = off) */
    double *d_stuck = nullptr;             /* [STUCK_CAP][STUCK_WORDS] abandoned-photon records */
    double *d_spec_blocks = nullptr;       /* per-workgroup spectrum slices */
    LoneRec *d_lone = nullptr;             /* photons handed over to lone_kernel */
    unsigned long long lone_cap = 0;
    int lone = 1;                          /* GRM_OPT_LONE */
    /* early hand-over of long photons to early_kernel on a second stream (GRM_OPT_EARLY_STEPS): 1,500
     * (~100 photons a bench pass) rather than 5,000 (~1): frozen-bias replays of the tail passes end
     * 14-48 ms sooner, the others unchanged; 1,000 fills the 1,024-slot queue */
    int early_steps = 1500;
    /* GRM_OPT_JOB_START_WAIT_MS: default 0.  Ranks of a real multi-GPU job run their passes back to back
     * without a host barrier between passes (bench.py), so a rank held up by a long photon would stall
     * every other rank's next warm-up; the one-GPU emulation of N ranks, whose launches queue behind
     * each other, sets it (tests/multirank_emu.py) */
    int64_t job_start_wait_ms = 0;
    /* The queue has EARLY_CAP slots, claimed once per launch.  The photons reaching S steps fall off
     * steeply with S (per 14.5 M-photon bench pass: ~680 at 1,200 steps, ~110 at 1,500, ~10 at
     * 2,000, ~1 at 5,000 -- about S^-8.5), so a call of many more photons (a configs[3] shard, 1.8e8
     * in one call) would fill the queue at 1,500 and keep its later long photons in the lane loop.
     * The threshold therefore grows with the call past 16 M photons as (n / 16 M)^(1/8.5): the same
     * expected hand-overs per call (~100-150) as a bench pass, 1,500 -> ~2,000 for a 1.8e8 shard. */
    static int early_steps_for(int base, size_t n) {
        const double ref = 16.0e6;
        if (base <= 0 || (double)n <= ref) return base;
        const double s = (double)base * std::pow((double)n / ref, 1.0 / 8.5);
        return s > (double)(1 << 30) ? (1 << 30) : (int)s;
    }
    bool early_serial = false; /* test: the worker ahead of the main launch on its stream */
    int early_children = 1;    /* GRM_OPT_EARLY_CHILDREN: the worker tracks its photons' children itself */
    int karg_test = 0;         /* test: GRM_OPT_KARG_TEST */
    static constexpr unsigned long long EARLY_CAP = 1024;
    LoneRec *d_early = nullptr;
    unsigned long long *d_early_ready = nullptr;
    /* the lone kernel's children queue (Ctl::lk_*): LK_CAP slots, their ready tags, and the five words
     * tail, taken, active, standby, originals finished (one per SMALL_STRIDE), cleared before every
     * lone launch */
    static constexpr unsigned long long LK_CAP = 4096;
    LoneRec *d_lk = nullptr;
    unsigned long long *d_lk_ready = nullptr, *d_lk_words = nullptr; /* words: 5 x SMALL_STRIDE */
    unsigned long long launch_seq = 0;
    size_t waves_rows = 0; /* rows of d_waves the last recorded launch wrote */
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_pre = nullptr, ev_w = nullptr;
    unsigned long long warmup_b0 = 64;     /* GRM_OPT_WARMUP_BATCH */
    /* GRM_OPT_WARMUP_SPREAD: 4 photons per wave claim spread a batch over 4-16x more waves, so the
     * families of its photons (the first photons' bias is large: long scattering cascades, each on
     * its wave's stack) get more lanes each -- the warm-up of a photon_n = 1e6 pass ends at ~28 ms
     * instead of ~49, recorded unchanged within 1.3 % (12 passes per setting, profiles/r03_ab/
     * r03p_warmup_spread_*.log; 1: 41 ms, 2: 32, 8: 29, 16: 31).  -1 (default) = auto: 4 for the
     * WARMUP_PHOTONS warm-up; none for the ramp to a grid of lanes (its batches outnumber the
     * warm-up's lanes) */
    int64_t warmup_spread = -1;
    /* host-mapped control block: ctl_kernel mirrors the counters and the small words here (ctr,
     * small) and the emission scan writes its total (word[4]); the host reads them after a stream
     * synchronisation, so a pass runs without copy or fill kernels (see ctl_kernel) */
    struct Pinned {
        DevCounters ctr;
        unsigned long long small[16];
        unsigned long long word[8];
    } *pin = nullptr;
    /* device emission: zone table, emission tables, zone offsets, emitted photons */
    grm_emit_zone *d_ezones = nullptr;
    double *d_eweight = nullptr, *d_ef = nullptr;
    unsigned long long *d_eoff = nullptr;
    int64_t n_ezones = 0;
    grm_init_photon *d_emit = nullptr;
    size_t emit_cap = 0;
    std::string err;
};

namespace {

bool hip_ok(grm_engine *e, hipError_t st, const char *what) {
    if (st == hipSuccess) return true;
    if (e) e->err = std::string(what) + ": " + hipGetErrorString(st);
    return false;
}

#define HIPCHK(e, call)                                   \
    do {                                                  \
        if (!hip_ok((e), (call), #call)) return -1;       \
    } while (0)

/* one ctl_kernel launch on the engine stream (op: the words to set; the mirror is always made) */
int ctl(grm_engine *e, CtlOp op, bool sync) {
    op.ctr = e->d_ctr;
    op.small = e->d_small;
    op.h_ctr = &e->pin->ctr;
    op.h_small = e->pin->small;
    unsigned blocks = 1;
    if (op.reset) {
        op.spec = reinterpret_cast<double *>(e->d_spec);
        op.n_spec = sizeof(grm_spectrum_cell) / sizeof(double) * N_TH_BINS * N_E_BINS;
        blocks = (unsigned)((op.n_spec + 255) / 256);
        std::memcpy(&op.max_tau_init_bits, &e->max_tau_init, sizeof(double));
    }
    hipLaunchKernelGGL(ctl_kernel, dim3(blocks), dim3(256), 0, e->stream, op);
    HIPCHK(e, hipGetLastError());
    if (sync) HIPCHK(e, hipStreamSynchronize(e->stream));
    return 0;
}

/* the device counters, through the host-mapped mirror */
int read_counters(grm_engine *e, DevCounters &h) {
    if (ctl(e, CtlOp{}, true)) return -1;
    h = e->pin->ctr; /* written by the device before the synchronisation returned */
    return 0;
}

int alloc_lanes(grm_engine *e) {
    int n_cu = 0;
    HIPCHK(e, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, e->device));
    int per_cu = 0;
    HIPCHK(e, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, track_kernel, BLOCK, 0));
    if (per_cu < 1) per_cu = 1;
    int grid = e->grid_override > 0 ? e->grid_override : n_cu * per_cu;
    if (grid < 1) grid = 1;
    const size_t lanes = (size_t)grid * BLOCK;
    if (lanes != e->lanes) {
        if (e->d_stack) (void)hipFree(e->d_stack);
        if (e->d_cold) (void)hipFree(e->d_cold);
        e->d_stack = nullptr;
        e->d_cold = nullptr;
        HIPCHK(e, hipMalloc(&e->d_stack, lanes * STACK_DEPTH * sizeof(SReq)));
        HIPCHK(e, hipMalloc(&e->d_cold, lanes * sizeof(Cold)));
        if (e->d_waves) (void)hipFree(e->d_waves);
        e->d_waves = nullptr;
        /* + PHASE_LOG words: the launch's phase stamps (grm_engine_debug_phases / _admissions) */
        HIPCHK(e, hipMalloc(&e->d_waves, (lanes / 64 * 4 + PHASE_LOG) * sizeof(unsigned long long)));
        if (e->d_spec_blocks) (void)hipFree(e->d_spec_blocks);
        e->d_spec_blocks = nullptr;
        HIPCHK(e, hipMalloc(&e->d_spec_blocks, (size_t)grid * SPEC_LDS * sizeof(double)));
        HIPCHK(e, hipMemset(e->d_spec_blocks, 0, (size_t)grid * SPEC_LDS * sizeof(double)));
        /* at most one hand-over per wave per launch (one per lane and launch's photon in the test
         * mode GRM_OPT_LONE = 2, sized in run_passes) */
        if (e->d_lone) (void)hipFree(e->d_lone);
        e->d_lone = nullptr;
        e->lone_cap = lanes / 64;
        HIPCHK(e, hipMalloc(&e->d_lone, e->lone_cap * sizeof(LoneRec)));
        e->lanes = lanes;
    }
    e->grid = grid;
    return 0;
}

int ensure_ovf(grm_engine *e, unsigned long long cap) {
    if (cap <= e->ovf_cap) return 0;
    for (int i = 0; i < 2; ++i) {
        if (e->d_ovf[i]) hipFree(e->d_ovf[i]);
        e->d_ovf[i] = nullptr;
        HIPCHK(e, hipMalloc(&e->d_ovf[i], cap * sizeof(SReq)));
    }
    e->ovf_cap = cap;
    return 0;
}

/* Live-bias warm-up size (GRM_OPT_WARMUP = -2, the default).  The counters bias_func reads lag the
 * claims by the photons in flight (~lanes): while the history is short against that, photons start
 * on a bias the serial reference never had.  A call of fewer than WARMUP_AUTO_RATIO x lanes photons
 * (photon_n = 1e5 on one GPU: 11 x lanes) ramps admission until the history reaches a grid's worth
 * of lanes: recorded +6.1 % -> +1.8 % against the oracle at 192^2, photon_n = 1e5, for +73 ms per
 * pass (16 seeds, profiles/r03d_warmup_rank_sweep_1e5.log; 16 k and 64 k photons did not move it).
 * A larger call (the bench's photon_n = 1e6: 110 x lanes) keeps WARMUP_PHOTONS: its lag is ~1 % of
 * the pass, and the ramp would cost ~15 % of it. */
constexpr uint64_t WARMUP_AUTO_RATIO = 32, WARMUP_PHOTONS = 4096;
/* The barrier before each admission batch waits until in-flight <= history / 2^slack.  Slack 1
 * (1/2) instead of 4 (1/16) shortened a photon_n = 1e6 launch by ~30 ms, the recorded count within
 * the oracle's spread (17.6 / 17.0 M against 17.64 +- 0.55 M; profiles/r03_ab/r3k_*).  The
 * admission log (grm_engine_debug_admissions, profiles/r03_ab/r03o_*) then shows batches 2-7
 * opening within 0.3 ms and the end of the warm-up at ~48 ms: the last batch waits for the
 * scattering families of its photons (the first photons' bias is large), each on its own wave's
 * stack -- hence WARMUP_SPREAD photons per wave claim (~28 ms).  The ramp of small passes (above)
 * keeps 1/16: there the history it builds is the point. */
constexpr int WARMUP_SLACK_LARGE = 1;
constexpr unsigned long long WARMUP_SPREAD = 4;

/* one launch (+ overflow relaunches) over claim positions [pos0, pos1) of a batch of n primaries
 * interleaved as 2^sh runs of m (Ctl.pos_end) */
int run_passes(grm_engine *e, const grm_init_photon *d_batch, size_t n, int sh, uint64_t m, uint64_t pos0,
               uint64_t pos1, int grid) {
    if (pos1 <= pos0) return 0;
    /* overflow pool: children rarely spill (a 1,024-deep stack per wave): a few hundred per
     * photon_n = 1e6 pass, 213-238 for the 1.8e8-photon shard of BASELINE configs[3]; size
     * max(1M, n/32) -- 2 x 1.1 GB for that shard, so eight such engines fit one GPU (n/4 took
     * 2 x 8.8 GB each).  A child that fits nowhere is counted and fails the call (n_dropped). */
    if (ensure_ovf(e, std::max<unsigned long long>(1ull << 20, (pos1 - pos0) / 32))) return -1;
    if (e->lone == 2 && e->lone_cap < e->ovf_cap + n) { /* test mode: every photon may be handed over */
        if (e->d_lone) (void)hipFree(e->d_lone);
        e->d_lone = nullptr;
        e->lone_cap = e->ovf_cap + n;
        HIPCHK(e, hipMalloc(&e->d_lone, e->lone_cap * sizeof(LoneRec)));
    }
    Ctl C{};
    C.pool = d_batch;
    C.pool_kind = 0;
    C.n_pool = n;
    C.pos_end = pos1;
    C.pool_m = m;
    C.pool_sh = sh;
    C.pool_head = e->d_small + (0) * SMALL_STRIDE;
    C.id_base = e->id_base;
    C.key0 = (uint32_t)e->seed;
    C.key1 = (uint32_t)(e->seed >> 32);
    C.stack = e->d_stack;
    C.cold = e->d_cold;
    C.ovf_cap = e->ovf_cap;
    C.spec = e->d_spec;
    C.spec_blocks = e->d_spec_blocks;
    C.ctr = e->d_ctr;
    C.peers = e->d_peers;
    C.n_peers = (e->ctr_slot >= 0 && e->d_peers) ? e->n_peers : 0;
    C.ctr_slot = e->ctr_slot;
    C.trace = e->trace_cap ? e->d_trace : nullptr;
    C.trace_cap = e->trace_cap;
    C.trace_count = e->d_small + (3) * SMALL_STRIDE;
    C.timing = e->d_timing;
    C.refill_min = e->refill_min;
    C.child_min = e->child_min;
    C.lanes = (int)e->lanes;
    C.bias_frozen = e->bias_mode;
    /* a multi-rank job's flight goes to the pass block, where the other ranks' gates read it */
    C.in_flight = C.n_peers > 1 ? &e->d_ctr->warm : e->d_small + (4) * SMALL_STRIDE;
    C.admit_end = e->d_small + (5) * SMALL_STRIDE;
    C.watchdog_ticks = (unsigned long long)std::max<int64_t>(e->watchdog_ms, 0) * 100000ull; /* 100 MHz */
    C.start_wait_ticks = (unsigned long long)e->job_start_wait_ms * 100000ull;
    C.stuck = e->d_stuck;
    C.stuck_cap = STUCK_CAP;
    C.stuck_count = e->d_small + (6) * SMALL_STRIDE;
    C.lone = e->lone ? e->d_lone : nullptr;
    C.lone_cap = e->lone_cap;
    C.lone_count = e->d_small + (7) * SMALL_STRIDE;
    C.lone_all = e->lone == 2;
    C.karg_test = e->karg_test;
    C.split_thr = e->split_thr;
    C.split_spin = e->split_spin;
    C.split_gthr = e->split_gthr;
    C.split_mode = e->split;
    C.split_batch = e->split_batch;
    {
        /* live-bias warm-up (GRM_OPT_WARMUP): the first photons after a reset start as the
         * counters' history doubles, as the serial reference's bias_func sees them */
        const uint64_t n_call = pos1 - pos0;
        const uint64_t lanes = (uint64_t)grid * BLOCK; /* this call's launch */
        const bool small = n_call < WARMUP_AUTO_RATIO * lanes;
        const uint64_t limit = e->warmup == -2 ? (small ? lanes : WARMUP_PHOTONS)
                               : e->warmup < 0 ? lanes
                                               : (uint64_t)e->warmup;
        /* a multi-rank job ramps the job's history to n_peers x one GPU's warm-up (see the kernel) */
        const uint64_t lim = C.n_peers > 1 ? limit * (uint64_t)C.n_peers : limit;
        C.admit_n = (!e->bias_mode && e->history < lim && pos0 == 0) ? std::min<uint64_t>(pos1, lim - e->history) : 0;
        C.admit_h0 = e->history;
        C.admit_lim = lim;
        /* slack: 1/16 for the small-call ramp and for a multi-rank job (its ranks' batches interleave
         * in 1/N shares; emulated 8-rank jobs, 48 each against the oracle at photon_n = 1e5: +4.1 to
         * +5.5 % recorded at 1/2 over five sessions, +2.3 / +2.4 / +3.1 % at 1/16 with warm-ups of 4 k /
         * 16 k / 64 k photons per rank, profiles/r04r_emu_sweep.log, r04y_emu.log) */
        C.admit_slack = e->warmup_slack >= 0 ? e->warmup_slack
                                              : ((e->warmup == -2 && small) || C.n_peers > 1 ? 4 : WARMUP_SLACK_LARGE);
        /* With the job's counters (n_peers ranks), every rank ramps at once: its batches are 1/n_peers
         * of a single GPU's, so that the JOB admits 64, 64, 128, ... photons against the job-wide
         * history as one GPU does (each rank at full batches would start n_peers x 64 photons on the
         * empty history, and so on at every doubling) */
        C.admit_b0 = C.n_peers > 1 ? std::max<unsigned long long>(1ull, e->warmup_b0 / (unsigned long long)C.n_peers)
                                   : e->warmup_b0;
        C.admit_spread = e->warmup_spread >= 0 ? (unsigned long long)e->warmup_spread
                                               : (e->warmup == -2 && small ? 0ull : WARMUP_SPREAD);
    }
    if (e->bias_mode && e->frozen_set) {
        C.f_scatt = e->fz_scatt;
        C.f_rec = e->fz_rec;
        C.f_maxtau = e->fz_maxtau;
    } else if (e->bias_mode) {
        DevCounters h;
        if (read_counters(e, h)) return -1;
        C.f_scatt = (double)h.n_scatt;
        C.f_rec = (double)h.n_recorded;
        double mt;
        std::memcpy(&mt, &h.max_tau_bits, sizeof(mt));
        C.f_maxtau = mt;
    }
    unsigned long long steps_before = 0;
    {
        DevCounters h;
        if (read_counters(e, h)) return -1;
        steps_before = h.n_steps;
    }
    double ms_total = 0.0;
    unsigned long long steps_pass = steps_before;
    int src = -1, dst = 0;
    unsigned long long n_pool = pos1 - pos0;
    for (int pass = 0; n_pool > 0; ++pass) {
        /* the words this launch starts from: [0] pool head (the first claim position), [1 + dst] its
         * overflow count (and that of the pool it drains), [4] in flight and [5] the end of the first
         * warm-up batch, [7] hand-overs; the abort flag cleared */
        CtlOp op{};
        op.clear_abort = 1;
        op.set = (1u << 0) | (1u << 1) | (1u << 2) | (1u << 7);
        op.val[0] = pass == 0 ? pos0 : 0;
        if (pass == 0 && C.admit_n) {
            const unsigned long long h = C.admit_h0;
            op.set |= (1u << 4) | (1u << 5);
            op.val[4] = 0;
            const unsigned long long n_r = C.n_peers > 1 ? (unsigned long long)C.n_peers : 1ull;
            op.val[5] = std::min<unsigned long long>(C.admit_n, std::max<unsigned long long>(
                                                                    C.admit_b0, std::min(h, C.admit_lim - h) / n_r));
            /* the job's gate counts this rank's earlier calls as admitted history */
            op.set_warm = C.n_peers > 1;
            op.warm_val = h * WARM_HIST;
        }
        /* the main launch runs the early worker beside it: [8] early tail, [9] head, [10] done,
         * [11] workgroups exited, [12] worker running / closed, [13] bulk started, [14] slots
         * finished, [15] the worker's children in its queue */
        const bool early = pass == 0 && C.pool_kind == 0 && e->early_steps > 0 && !C.lone_all && grid > 1;
        if (early) op.set |= 0xff00u;
        if (ctl(e, op, false)) return -1;
        if (early) {
            C.early_q = e->d_early;
            C.early_ready = e->d_early_ready;
            C.early_cap = grm_engine::EARLY_CAP;
            C.early_tag = ++e->launch_seq;
            C.early_tail = e->d_small + (8) * SMALL_STRIDE;
            C.early_head = e->d_small + (9) * SMALL_STRIDE;
            C.early_done = e->d_small + (10) * SMALL_STRIDE;
            C.wg_exit = e->d_small + (11) * SMALL_STRIDE;
            C.early_live = e->d_small + (12) * SMALL_STRIDE;
            C.bulk_live = e->d_small + (13) * SMALL_STRIDE;
            C.early_steps = grm_engine::early_steps_for(e->early_steps, n);
            C.early_kids_on = e->early_children;
            C.early_fin = e->d_small + (14) * SMALL_STRIDE;
            C.early_kids = e->d_small + (15) * SMALL_STRIDE;
        } else {
            C.early_q = nullptr;
            C.early_kids_on = 0;
        }
        C.ovf = e->d_ovf[dst];
        C.ovf_count = e->d_small + (1 + dst) * SMALL_STRIDE;
        /* the per-wave record is kept of the first launch (the bulk of a call) */
        C.waves = pass == 0 ? e->d_waves : nullptr;
        C.phases = C.waves ? e->d_waves + (size_t)(e->lanes / 64) * 4 : nullptr;
        if (C.phases) HIPCHK(e, hipMemsetAsync(C.phases, 0, PHASE_LOG * sizeof(unsigned long long), e->stream));
        if (C.waves) e->waves_rows = (size_t)grid * (BLOCK / 64);
        if (pass > 0) {
            C.pool = e->d_ovf[src];
            C.pool_kind = 1;
            C.n_pool = n_pool;
            C.pos_end = n_pool;
            C.pool_m = n_pool;
            C.pool_sh = 0;
            C.admit_n = 0;
            /* a small relaunch (the children of the hand-overs, a few hundred) is a tail from its
             * start: every photon goes to a two-wave pair at the top of its first step (~1.5 us per
             * step against ~4 us in a sparse lane loop) */
            C.lone_all = e->lone == 2 || (e->lone == 1 && n_pool <= e->lone_cap / 2);
        }
        if (early && e->early_serial) { /* test: serialised ahead of the main launch */
            HIPCHK(e, grm_lone_launch(1, 1, e->stream, &e->P, sizeof(Params), &C, sizeof(Ctl)));
            HIPCHK(e, hipEventRecord(e->ev_w, e->stream));
        } else if (early) { /* after the control words are set; one workgroup, all of its pairs */
            HIPCHK(e, hipEventRecord(e->ev_pre, e->stream));
            HIPCHK(e, hipStreamWaitEvent(e->stream2, e->ev_pre, 0));
            HIPCHK(e, grm_lone_launch(1, 1, e->stream2, &e->P, sizeof(Params), &C, sizeof(Ctl)));
            HIPCHK(e, hipEventRecord(e->ev_w, e->stream2));
        }
        HIPCHK(e, hipEventRecord(e->ev0, e->stream));
        /* one workgroup per CU.  The early worker takes one CU too: workgroups are dealt to the XCDs
         * round-robin, so with the worker's XCD full one bulk workgroup waits and starts (to find
         * the pool empty) as the bulk drains -- 255 run either way, and a full grid needs no guess
         * which XCD the worker lands on */
#ifdef GRM_WITH_SPLIT
        if (e->split) {
            HIPCHK(e, grm_split_launch((unsigned)grid, e->stream, &e->P, sizeof(Params), &C, sizeof(Ctl)));
        } else
#endif
        {
            hipLaunchKernelGGL(track_kernel, dim3(grid), dim3(BLOCK), 0, e->stream, e->P, C);
            HIPCHK(e, hipGetLastError());
        }
        HIPCHK(e, hipEventRecord(e->ev1, e->stream));
        /* the photons the launch handed over (a count on the device), one wave pair each; their
         * children join this launch's overflow pool */
        if (C.lone) {
            /* the lone pairs track the children of their photons themselves (GRM_OPT_EARLY_CHILDREN) */
            C.lk_on = e->early_children;
            C.lk_q = e->d_lk;
            C.lk_ready = e->d_lk_ready;
            C.lk_cap = grm_engine::LK_CAP;
            C.lk_tag = ++e->launch_seq;
            C.lk_tail = e->d_lk_words + 0 * SMALL_STRIDE;
            C.lk_taken = e->d_lk_words + 1 * SMALL_STRIDE;
            C.lk_active = e->d_lk_words + 2 * SMALL_STRIDE;
            C.lk_standby = e->d_lk_words + 3 * SMALL_STRIDE;
            C.lk_orig = e->d_lk_words + 4 * SMALL_STRIDE;
            if (C.lk_on)
                HIPCHK(e, hipMemsetAsync(e->d_lk_words, 0, 5 * SMALL_STRIDE * sizeof(unsigned long long), e->stream));
            HIPCHK(e, hipEventRecord(e->ev2, e->stream));
            HIPCHK(e, grm_lone_launch(0, (unsigned)e->lone_cap, e->stream, &e->P, sizeof(Params), &C, sizeof(Ctl)));
            HIPCHK(e, hipEventRecord(e->ev3, e->stream));
        }
        if (early) HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_w, 0)); /* its photons' counters too */
        DevCounters hp;
        if (read_counters(e, hp)) return -1; /* synchronises */
        float ms = 0.f;
        HIPCHK(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
        ms_total += ms;
        const unsigned long long n_lone = std::min<unsigned long long>(e->pin->small[7], e->lone_cap);
        if (early) { /* the published slots: hand-overs and the worker's own children */
            const unsigned long long kids = e->pin->small[15];
            e->stats.n_early += std::min<unsigned long long>(e->pin->small[8], grm_engine::EARLY_CAP) - kids;
            e->stats.n_early_children += kids;
        }
        if (early && !e->early_serial) { /* ev_pre (engine stream, before the bulk) .. ev_w (after the worker) */
            float ms_e = 0.f;
            HIPCHK(e, hipEventElapsedTime(&ms_e, e->ev_pre, e->ev_w));
            if (ms_e > e->stats.early_ms) e->stats.early_ms = ms_e;
        }
        if (C.lone) {
            float ms_l = 0.f;
            HIPCHK(e, hipEventElapsedTime(&ms_l, e->ev2, e->ev3));
            ms_total += ms_l;
            e->stats.lone_ms += ms_l;
            e->stats.n_lone += n_lone;
            if (C.lk_on) {
                unsigned long long lk_tail = 0;
                HIPCHK(e, hipMemcpy(&lk_tail, e->d_lk_words, sizeof(lk_tail), hipMemcpyDeviceToHost));
                e->stats.n_lone_children += std::min<unsigned long long>(lk_tail, grm_engine::LK_CAP);
            }
            if (n_lone) e->stats.n_launches++;
        }
        const unsigned long long cnt = e->pin->small[1 + dst];
        if (ms > e->stats.max_launch_ms) { /* the dominant launch of this transport call */
            e->stats.max_launch_ms = ms;
            e->stats.max_launch_steps = hp.n_steps - steps_pass;
        }
        steps_pass = hp.n_steps;
        e->stats.n_launches++;
        e->stats.n_nan_photons = hp.n_nan;
        if (hp.karg_bad) {
            e->err = "track_kernel: the kernel-argument segment does not hold the launch's arguments in the "
                     "layout of struct KArgs (" + std::to_string(hp.karg_bad) +
                     " waves); no photon was tracked -- results of this call are invalid";
            return -1;
        }
        if (hp.abort) {
            e->stats.n_abandoned = hp.n_abandoned;
            e->err = "watchdog: a transport launch ran longer than " + std::to_string(e->watchdog_ms) + " ms; " +
                     std::to_string(hp.n_abandoned) +
                     " photons abandoned (their state: grm_engine_debug_stuck); results of this call are incomplete";
            return -1;
        }
        n_pool = std::min(cnt, e->ovf_cap);
        src = dst;
        dst ^= 1;
        if (pass > 64) {
            e->err = "overflow relaunch did not converge";
            return -1;
        }
    }
    DevCounters h;
    if (read_counters(e, h)) return -1;
    if (h.n_dropped) {
        /* a scattered child that fit neither the wave stack nor the overflow pool is lost: the
         * spectrum of this call would be incomplete, so the call fails */
        e->err = std::to_string(h.n_dropped) + " scattered children dropped (overflow pool of " +
                 std::to_string(e->ovf_cap) + " full); results of this call are incomplete";
        return -1;
    }
    e->stats.kernel_ms += ms_total;
    e->stats.last_kernel_ms += ms_total;
    e->stats.last_steps += h.n_steps - steps_before;
    e->history += pos1 - pos0;
    return 0;
}

/* One transport call = one persistent launch (+ overflow relaunches); the live-bias warm-up is
 * admission control inside the launch (Ctl.admit_n).
 *
 * Claim order.  The batch is in zone-walk order (emission, harm_model.cpp:673-704), and the
 * adaptive bias (bias_func, :1391-1404) is driven by the counters of RECORDED photons.  The inner
 * zones' photons fall into the hole and never record, so a zone-ordered claim sequence would start
 * ~lanes photons of the zones where escape begins all at once on the bias of an empty history --
 * where the serial reference adapts after the first few records -- and their scattering cascades
 * would inflate the recorded / scattered counts ~2x (measured: 5.1 M vs the reference's 2.3 M at
 * 192^2, photon_n = 1e5).  Claims therefore interleave 2^CLAIM_SH evenly spaced runs of the batch:
 * claim position q takes photon (q mod 2^CLAIM_SH) * m + q / 2^CLAIM_SH, so every admission batch
 * and every stretch of the bulk samples the whole zone range, records start at once and the
 * counters evolve as in the serial run (photon ids, and so the Philox streams, stay the batch
 * index: results depend on the order only through the bias). */
constexpr int CLAIM_SH = 12;

int run_transport(grm_engine *e, const grm_init_photon *d_batch, size_t n) {
    if (alloc_lanes(e)) return -1;
    e->stats.last_kernel_ms = 0.0;
    e->stats.last_steps = 0;
    e->stats.max_launch_ms = 0.0;
    e->stats.max_launch_steps = 0;
    if (n == 0) return 0;
    const int sh = n >= (2ull << CLAIM_SH) ? CLAIM_SH : 0;
    const uint64_t m = (n + (1ull << sh) - 1) >> sh, n_pos = m << sh;
    /* one launch: the live-bias warm-up (the first positions in admission batches) is admission
     * control inside it, and the claims run free as soon as it is over, while the warm-up's own
     * long-lived photons are still in flight.  With the live bias the launch has at most
     * n / flight_ratio lanes (GRM_OPT_FLIGHT_RATIO): the counters bias_func reads trail the claims
     * by the photons in flight, and a call of 1.45 M photons (photon_n = 1e5) on 131 k lanes moved
     * recorded / scattered / steps +4.4 / +5.9 / +4.2 % against the serial reference, +1.0 / +1.1 /
     * +0.9 % on 16 k lanes (96 seeds each, profiles/r04h_grid_sweep96.jsonl) -- for 1.6x the pass
     * time at that size; a bench pass (14.5 M photons) keeps the full grid.  The lag matters against
     * the history the counters already hold, so the cap counts the photons tracked since the reset
     * too: a pass fed in chunks (INTEGRATION.md path (a), 4 M photons per call) runs its later
     * chunks on the full grid */
    int grid = e->grid;
    if (!e->bias_mode && e->flight_ratio > 0) {
        /* A multi-rank job's small calls run on half those lanes: with the job's counters the ranks'
         * concurrent launches lag the job's history more than one GPU's launch with as many lanes
         * (emulated 8-rank jobs at photon_n = 1e5, 96 each, the same seeds: recorded +2.97 % at ratio
         * 96, +1.42 % at 192; one GPU +1.00 / +0.92 %, the serial reference on the same streams +0.85 %;
         * DESIGN.md §7).  Large calls (>= WARMUP_AUTO_RATIO x the full grid's lanes: the bench's 1e6
         * per rank, a configs[3] shard) keep the ratio, so the cap does not bind there. */
        const bool job = e->ctr_slot >= 0 && e->d_peers && e->n_peers > 1;
        const uint64_t full = (uint64_t)e->grid * BLOCK;
        const uint64_t ratio = (uint64_t)e->flight_ratio * ((job && e->history + n < WARMUP_AUTO_RATIO * full) ? 2 : 1);
        const uint64_t cap_wg = (e->history + n) / (ratio * BLOCK);
        grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)grid, cap_wg));
    }
    e->stats.last_grid = grid;
    if (run_passes(e, d_batch, n, sh, m, 0, n_pos, grid)) return -1;
    e->id_base += n;
    return 0;
}

int reset_counters(grm_engine *e) {
    CtlOp op{};
    op.reset = 1;
    op.set = 0xffffu; /* every small word 0 */
    return ctl(e, op, true);
}

} /* namespace */

/* probe entry point lives in grm_probe.hip */
extern "C" int grm_probe_impl(const Params &P, hipStream_t s, int which, const double *in, int in_stride, double *out,
                              int out_stride, size_t n, std::string &err);

extern "C" {

int grm_engine_create(const grm_header *h, const double *const fields[8], const grm_units *u, const double *hotcross,
                      const double *k2, const double scalars[4], int device, grm_engine **out) {
    if (!h || !fields || !u || !hotcross || !k2 || !scalars || !out) return -1;
    *out = nullptr;
    if (h->n[0] < 2 || h->n[1] < 2) return -2;
    grm_engine *e = new grm_engine();
    e->device = device;
    auto fail = [&](void) {
        *out = e; /* hand back for last_error; caller destroys */
        return -1;
    };
    if (!hip_ok(e, hipSetDevice(device), "hipSetDevice")) return fail();
    if (!hip_ok(e, hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking), "stream")) return fail();
    if (!hip_ok(e, hipEventCreate(&e->ev0), "event") || !hip_ok(e, hipEventCreate(&e->ev1), "event") ||
        !hip_ok(e, hipEventCreate(&e->ev2), "event") || !hip_ok(e, hipEventCreate(&e->ev3), "event") ||
        !hip_ok(e, hipEventCreate(&e->ev_pre), "event") || /* timed: stats.early_ms */
        !hip_ok(e, hipEventCreate(&e->ev_w), "event") ||
        !hip_ok(e, hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking), "stream") ||
        !hip_ok(e, hipMalloc(&e->d_early, grm_engine::EARLY_CAP * sizeof(LoneRec)), "early queue") ||
        !hip_ok(e, hipMalloc(&e->d_early_ready, grm_engine::EARLY_CAP * sizeof(unsigned long long)), "early queue") ||
        !hip_ok(e, hipMemset(e->d_early_ready, 0, grm_engine::EARLY_CAP * sizeof(unsigned long long)), "early queue") ||
        !hip_ok(e, hipMalloc(&e->d_lk, grm_engine::LK_CAP * sizeof(LoneRec)), "lone children queue") ||
        !hip_ok(e, hipMalloc(&e->d_lk_ready, grm_engine::LK_CAP * sizeof(unsigned long long)), "lone children queue") ||
        !hip_ok(e, hipMemset(e->d_lk_ready, 0, grm_engine::LK_CAP * sizeof(unsigned long long)), "lone children queue") ||
        !hip_ok(e, hipMalloc(&e->d_lk_words, 5 * SMALL_STRIDE * sizeof(unsigned long long)), "lone children queue"))
        return fail();
    if (!hip_ok(e, hipHostMalloc(reinterpret_cast<void **>(&e->pin), sizeof(grm_engine::Pinned),
                                 hipHostMallocMapped | hipHostMallocCoherent),
                "host-mapped control block"))
        return fail();
    std::memset(e->pin, 0, sizeof(grm_engine::Pinned));
    {
        /* the kernels write the block through the host pointer: it must be the device address too */
        void *dp = nullptr;
        if (!hip_ok(e, hipHostGetDevicePointer(&dp, e->pin, 0), "hipHostGetDevicePointer")) return fail();
        if (dp != (void *)e->pin) {
            e->err = "host-mapped control block: device address differs from the host address";
            return fail();
        }
    }
    const size_t nz = (size_t)h->n[0] * h->n[1];
    std::vector<double> zones(nz * 8);
    for (size_t z = 0; z < nz; ++z)
        for (int f = 0; f < 8; ++f) zones[z * 8 + f] = fields[f][z];
    const size_t nhot = (size_t)(GRM_HC_N_W + 1) * (GRM_HC_N_T + 1);
    if (!hip_ok(e, hipMalloc(&e->d_zones, nz * 8 * sizeof(double)), "zones") ||
        !hip_ok(e, hipMalloc(&e->d_hot, nhot * sizeof(double)), "hotcross") ||
        !hip_ok(e, hipMalloc(&e->d_k2, (GRM_N_E_SAMP + 1) * sizeof(double)), "k2") ||
        !hip_ok(e, hipMalloc(&e->d_ctr_own, sizeof(DevCounters)), "counters") ||
        !hip_ok(e, hipMalloc(&e->d_spec, sizeof(grm_spectrum_cell) * N_TH_BINS * N_E_BINS), "spectrum") ||
        !hip_ok(e, hipMalloc(&e->d_small, 16 * SMALL_STRIDE * sizeof(unsigned long long)), "small") ||
        !hip_ok(e, hipMalloc(&e->d_stuck, STUCK_CAP * STUCK_WORDS * sizeof(double)), "stuck") ||
        !hip_ok(e, hipMemset(e->d_small, 0, 16 * SMALL_STRIDE * sizeof(unsigned long long)), "small"))
        return fail();
    if (!hip_ok(e, hipMemcpy(e->d_zones, zones.data(), nz * 8 * sizeof(double), hipMemcpyHostToDevice), "H2D") ||
        !hip_ok(e, hipMemcpy(e->d_hot, hotcross, nhot * sizeof(double), hipMemcpyHostToDevice), "H2D") ||
        !hip_ok(e, hipMemcpy(e->d_k2, k2, (GRM_N_E_SAMP + 1) * sizeof(double), hipMemcpyHostToDevice), "H2D"))
        return fail();
    Params &P = e->P;
    P.n1 = h->n[0];
    P.n2 = h->n[1];
    P.xs1 = h->x_start[1];
    P.xs2 = h->x_start[2];
    P.xe1 = h->x_stop[1];
    P.xe2 = h->x_stop[2];
    P.dx1 = h->dx[1];
    P.dx2 = h->dx[2];
    P.a = h->a;
    P.h_slope = h->h_slope;
    P.r0 = h->r_0;
    P.n_e_unit = u->n_e_unit;
    P.theta_e_unit = u->theta_e_unit;
    P.b_unit = u->b_unit;
    P.bias_norm = scalars[0];
    P.x1_min = scalars[1];
    e->max_tau_init = scalars[2];
    P.d_tau_k = scalars[3];
    /* derived table constants, host libm (consts.hpp:33-157) */
    P.x1_max = std::log(100.0);
    P.hc_l_min_w = std::log10(1.0e-12);
    P.hc_l_min_t = std::log10(1.0e-4);
    P.hc_d_l_w = std::log10(1.0e6 / 1.0e-12) / GRM_HC_N_W;
    P.hc_d_l_t = std::log10(1.0e4 / 1.0e-4) / GRM_HC_N_T;
    P.jnu_l_min_t = std::log(0.3);
    P.jnu_d_l_t = std::log(1.0e2 / 0.3) / GRM_N_E_SAMP;
    P.spec_l_e_0 = std::log(1.0e-12);
    P.th_dx2 = (h->x_stop[2] - h->x_start[2]) / (2.0 * N_TH_BINS);
    P.i_dx1 = 1.0 / P.dx1;
    P.i_dx2 = 1.0 / P.dx2;
    P.hc_i_d_l_w = 1.0 / P.hc_d_l_w;
    P.hc_i_d_l_t = 1.0 / P.hc_d_l_t;
    P.jnu_i_d_l_t = 1.0 / P.jnu_d_l_t;
    params_metric(P);
    P.zones = e->d_zones;
    P.hotcross = e->d_hot;
    P.k2 = e->d_k2;
    e->d_ctr = e->d_ctr_own;
    if (!hip_ok(e, hipMalloc(&e->d_timing, 48 * sizeof(unsigned long long)), "timing") ||
        !hip_ok(e, hipMemset(e->d_timing, 0, 48 * sizeof(unsigned long long)), "timing"))
        return fail();
    if (reset_counters(e)) return fail();
    *out = e;
    return 0;
}

void grm_engine_destroy(grm_engine *e) {
    if (!e) return;
    hipSetDevice(e->device);
    if (e->stream) hipStreamSynchronize(e->stream);
    if (e->stream2) hipStreamSynchronize(e->stream2); /* early_kernel uses d_small, d_ctr, d_early ... */
    hipFree(e->d_zones);
    hipFree(e->d_hot);
    hipFree(e->d_k2);
    hipFree(e->d_ctr_own);
    for (void *p : e->ipc_open) hipIpcCloseMemHandle(p);
    hipFree(e->d_ctr_slots);
    hipFree(e->d_peers);
    hipFree(e->d_spec);
    hipFree(e->d_stack);
    hipFree(e->d_cold);
    hipFree(e->d_ovf[0]);
    hipFree(e->d_ovf[1]);
    hipFree(e->d_small);
    hipFree(e->d_stuck);
    hipFree(e->d_spec_blocks);
    hipFree(e->d_lone);
    if (e->pin) hipHostFree(e->pin);
    hipFree(e->d_batch);
    hipFree(e->d_trace);
    hipFree(e->d_upload);
    hipFree(e->d_timing);
    hipFree(e->d_waves);
    hipFree(e->d_ezones);
    hipFree(e->d_eweight);
    hipFree(e->d_ef);
    hipFree(e->d_eoff);
    hipFree(e->d_emit);
    if (e->comm) ncclCommDestroy(e->comm);
    hipFree(e->d_stash_spec);
    hipFree(e->d_stash_sum);
    hipFree(e->d_stash_max);
    if (e->ev0) hipEventDestroy(e->ev0);
    if (e->ev1) hipEventDestroy(e->ev1);
    if (e->ev2) hipEventDestroy(e->ev2);
    if (e->ev3) hipEventDestroy(e->ev3);
    if (e->ev_pre) hipEventDestroy(e->ev_pre);
    if (e->ev_w) hipEventDestroy(e->ev_w);
    if (e->stream2) hipStreamDestroy(e->stream2);
    hipFree(e->d_early);
    hipFree(e->d_early_ready);
    hipFree(e->d_lk);
    hipFree(e->d_lk_ready);
    hipFree(e->d_lk_words);
    if (e->stream) hipStreamDestroy(e->stream);
    delete e;
}

const char *grm_engine_last_error(const grm_engine *e) { return e ? e->err.c_str() : "null engine"; }

int grm_engine_set_option(grm_engine *e, int opt, int64_t v) {
    if (!e) return -1;
    hipSetDevice(e->device);
    switch (opt) {
    case GRM_OPT_SEED: e->seed = (uint64_t)v; return 0;
    case GRM_OPT_BIAS_MODE: e->bias_mode = v ? 1 : 0; return 0;
    case GRM_OPT_TRACE_CAP:
        if (e->d_trace) hipFree(e->d_trace);
        e->d_trace = nullptr;
        e->trace_cap = 0;
        if (v > 0) {
            HIPCHK(e, hipMalloc(&e->d_trace, (size_t)v * sizeof(grm_trace)));
            e->trace_cap = (unsigned long long)v;
        }
        return 0;
    case GRM_OPT_GRID_BLOCKS: e->grid_override = (int)v; return 0;
    case GRM_OPT_FLIGHT_RATIO: e->flight_ratio = v < 0 ? 0 : v; return 0;
    case GRM_OPT_JOB_START_WAIT_MS: e->job_start_wait_ms = v < 0 ? 0 : (v > 10000 ? 10000 : v); return 0;
    case GRM_OPT_ID_BASE: e->id_base = (uint64_t)v; return 0;
    case GRM_OPT_FROZEN_SCATT: e->fz_scatt = (double)v; e->frozen_set = true; return 0;
    case GRM_OPT_FROZEN_REC: e->fz_rec = (double)v; e->frozen_set = true; return 0;
    case GRM_OPT_FROZEN_MAXTAU: std::memcpy(&e->fz_maxtau, &v, sizeof(double)); e->frozen_set = true; return 0;
    case GRM_OPT_WARMUP: e->warmup = v; return 0;
    case GRM_OPT_REFILL_MIN: e->refill_min = v < 1 ? 1 : (v > 64 ? 64 : (int)v); return 0;
    case GRM_OPT_CHILD_MIN: e->child_min = v < 1 ? 1 : (v > 64 ? 64 : (int)v); return 0;
    case GRM_OPT_WARMUP_SLACK: e->warmup_slack = v < 0 ? -1 : (v > 30 ? 30 : (int)v); return 0;
    case GRM_OPT_LONE: e->lone = v < 0 ? 0 : (v > 2 ? 2 : (int)v); return 0;
    case GRM_OPT_WARMUP_BATCH: e->warmup_b0 = v < 1 ? 1 : (unsigned long long)v; return 0;
    case GRM_OPT_WARMUP_SPREAD: e->warmup_spread = v < 0 ? -1 : v; return 0;
    case GRM_OPT_EARLY_STEPS: e->early_steps = v < 0 ? 0 : (v > (1 << 30) ? (1 << 30) : (int)v); return 0;
    case GRM_OPT_EARLY_SERIAL: e->early_serial = v != 0; return 0;
    case GRM_OPT_EARLY_CHILDREN: e->early_children = v != 0; return 0;
    case GRM_OPT_KARG_TEST: e->karg_test = (int)v; return 0;
    case GRM_OPT_WATCHDOG_MS: e->watchdog_ms = v < 0 ? 0 : v; return 0;
#ifdef GRM_WITH_SPLIT
    case GRM_OPT_SPLIT: e->split = v < 0 ? 0 : (v > 2 ? 2 : (int)v); return 0;
    case GRM_OPT_SPLIT_THR: e->split_thr = v < 1 ? 1 : (v > 64 ? 64 : (int)v); return 0;
    case GRM_OPT_SPLIT_SPIN: e->split_spin = v < 0 ? 0 : (v > 1 << 20 ? 1 << 20 : (int)v); return 0;
    case GRM_OPT_SPLIT_GTHR: e->split_gthr = v < 0 ? 0 : (v > 64 ? 64 : (int)v); return 0;
    case GRM_OPT_SPLIT_BATCH: e->split_batch = v < 1 ? 1 : (v > 3 ? 3 : (int)v); return 0;
#else
    case GRM_OPT_SPLIT:
        if (v == 0) return 0; /* track_kernel: the only bulk kernel of this build */
        e->err = "split_kernel is not in this library (a variant build: VFLAGS=-DGRM_WITH_SPLIT tools/build_variant.sh)";
        return -1;
    case GRM_OPT_SPLIT_THR: case GRM_OPT_SPLIT_SPIN: case GRM_OPT_SPLIT_GTHR: case GRM_OPT_SPLIT_BATCH:
        e->err = "split_kernel options need a variant build with -DGRM_WITH_SPLIT";
        return -1;
#endif
    case 18: case 20: case 21: e->err = "retired option " + std::to_string(opt); return -1;
    default: e->err = "unknown option"; return -1;
    }
}

int grm_engine_track(grm_engine *e, const grm_init_photon *batch, size_t n) {
    if (!e || (!batch && n)) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    if (n > e->batch_cap) { /* 1/8 headroom, as the emission buffer (grm_emit.hip) */
        if (e->d_batch) hipFree(e->d_batch);
        e->d_batch = nullptr;
        HIPCHK(e, hipMalloc(&e->d_batch, (n + n / 8) * sizeof(grm_init_photon)));
        e->batch_cap = n + n / 8;
    }
    HIPCHK(e, hipMemcpyAsync(e->d_batch, batch, n * sizeof(grm_init_photon), hipMemcpyHostToDevice, e->stream));
    return run_transport(e, e->d_batch, n);
}

int grm_engine_track_device(grm_engine *e, const grm_init_photon *dev_batch, size_t n) {
    if (!e || (!dev_batch && n)) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    return run_transport(e, dev_batch, n);
}

int grm_engine_finish(grm_engine *e, grm_spectrum_cell *spec, uint64_t *n_rec, uint64_t *n_scatt, double *max_tau) {
    if (!e) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    DevCounters h;
    if (spec)
        HIPCHK(e, hipMemcpyAsync(spec, e->d_spec, sizeof(grm_spectrum_cell) * N_TH_BINS * N_E_BINS,
                                 hipMemcpyDeviceToHost, e->stream));
    if (read_counters(e, h)) return -1;
    if (n_rec) *n_rec = h.n_recorded;
    if (n_scatt) *n_scatt = h.n_scatt;
    if (max_tau) std::memcpy(max_tau, &h.max_tau_bits, sizeof(double));
    e->stats.n_steps = h.n_steps;
    e->stats.n_tracked = h.n_tracked;
    e->stats.n_children = h.n_children;
    e->stats.n_overflow = h.n_overflow;
    e->stats.n_dropped = h.n_dropped;
    e->stats.n_primaries = h.n_primaries;
    e->stats.max_photon_steps = h.max_nstep;
    e->stats.n_long_photons = h.n_long;
    return 0;
}

int grm_engine_reset(grm_engine *e) {
    if (!e) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    const double ms = e->stats.kernel_ms;
    const uint64_t launches = e->stats.n_launches;
    std::memset(&e->stats, 0, sizeof(e->stats));
    e->stats.kernel_ms = ms;
    e->stats.n_launches = launches;
    e->history = 0;
    return reset_counters(e);
}

int grm_engine_stats(const grm_engine *e, grm_stats *out) {
    if (!e || !out) return -1;
    grm_engine *m = const_cast<grm_engine *>(e);
    if (grm_engine_finish(m, nullptr, nullptr, nullptr, nullptr)) return -1;
    *out = e->stats;
    return 0;
}

void *grm_engine_spectrum_device_ptr(grm_engine *e) { return e ? (void *)e->d_spec : nullptr; }

int64_t grm_engine_trace(grm_engine *e, grm_trace *out, size_t cap) {
    if (!e || !e->d_trace) return -1;
    hipSetDevice(e->device);
    unsigned long long cnt = 0;
    if (hipMemcpy(&cnt, e->d_small + (3) * SMALL_STRIDE, sizeof(cnt), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    const size_t avail = std::min<unsigned long long>(cnt, e->trace_cap);
    const size_t k = std::min(avail, cap);
    if (k && out && hipMemcpy(out, e->d_trace, k * sizeof(grm_trace), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (int64_t)cnt;
}

int grm_engine_upload(grm_engine *e, const grm_init_photon *batch, size_t n, grm_init_photon **dev_out) {
    if (!e || !dev_out || (!batch && n)) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    if (n > e->upload_cap) {
        if (e->d_upload) (void)hipFree(e->d_upload);
        e->d_upload = nullptr;
        e->upload_cap = 0;
        HIPCHK(e, hipMalloc(&e->d_upload, n * sizeof(grm_init_photon)));
        e->upload_cap = n;
    }
    HIPCHK(e, hipMemcpy(e->d_upload, batch, n * sizeof(grm_init_photon), hipMemcpyHostToDevice));
    *dev_out = e->d_upload;
    return 0;
}

int grm_engine_emit_setup(grm_engine *e, const grm_emit_zone *zones, int64_t n_zones, const double *weight,
                          const double *f) {
    if (!e) return -1;
    if (!zones || !weight || !f || n_zones != (int64_t)e->P.n1 * e->P.n2) {
        e->err = "grm_engine_emit_setup: need the zone table of all n1*n2 zones and both emission tables";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    hipFree(e->d_ezones);
    hipFree(e->d_eweight);
    hipFree(e->d_ef);
    hipFree(e->d_eoff);
    e->d_ezones = nullptr;
    e->d_eweight = e->d_ef = nullptr;
    e->d_eoff = nullptr;
    e->n_ezones = 0;
    const size_t nt = GRM_N_E_SAMP + 1;
    HIPCHK(e, hipMalloc(&e->d_ezones, (size_t)n_zones * sizeof(grm_emit_zone)));
    HIPCHK(e, hipMalloc(&e->d_eweight, nt * sizeof(double)));
    HIPCHK(e, hipMalloc(&e->d_ef, nt * sizeof(double)));
    HIPCHK(e, hipMalloc(&e->d_eoff, ((size_t)n_zones + 1) * sizeof(unsigned long long)));
    HIPCHK(e, hipMemcpy(e->d_ezones, zones, (size_t)n_zones * sizeof(grm_emit_zone), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_eweight, weight, nt * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_ef, f, nt * sizeof(double), hipMemcpyHostToDevice));
    e->n_ezones = n_zones;
    return 0;
}

int grm_engine_emit(grm_engine *e, uint64_t seed, int64_t z0, int64_t z1, grm_init_photon **dev_out,
                    uint64_t *n_out) {
    return grm_engine_emit_strided(e, seed, z0, z1, 1, dev_out, n_out);
}

int grm_engine_emit_strided(grm_engine *e, uint64_t seed, int64_t z0, int64_t z1, int64_t stride,
                            grm_init_photon **dev_out, uint64_t *n_out) {
    if (!e || !dev_out || !n_out) return -1;
    if (stride < 1) {
        e->err = "grm_engine_emit_strided: stride < 1";
        return -1;
    }
    if (!e->d_ezones) {
        e->err = "grm_engine_emit: no zone table (grm_engine_emit_setup)";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    if (z1 < 0 || z1 > e->n_ezones) z1 = e->n_ezones;
    if (z0 < 0) z0 = 0;
    if (z0 > z1) z0 = z1;
    const uint64_t n_zones = (uint64_t)((z1 - z0 + stride - 1) / stride);
    /* consts.hpp:33-157 emission constants, host libm like the host model's */
    EmitParams E;
    E.zones = e->d_ezones;
    E.weight = e->d_eweight;
    E.f = e->d_ef;
    E.l_nu_min = std::log(1.0e9);
    const double l_nu_max = std::log(1.0e16);
    E.n_l_n = l_nu_max - E.l_nu_min;
    E.d_l_nu = (l_nu_max - E.l_nu_min) / GRM_N_E_SAMP;
    E.jnu_l_min_k = std::log(0.002);
    E.jnu_d_l_k = std::log(1.0e7 / 0.002) / GRM_N_E_SAMP;
    E.k0 = (uint32_t)seed;
    E.k1 = (uint32_t)(seed >> 32);
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    uint64_t n = 0;
    if (grm_emit_launch(e->P, E, (uint64_t)z0, (uint64_t)stride, n_zones, e->d_eoff, e->stream, &e->pin->word[4], &e->d_emit,
                        &e->emit_cap, &n, e->err))
        return -1;
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipEventSynchronize(e->ev1));
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
    e->stats.last_emit_ms = ms;
    *dev_out = e->d_emit;
    *n_out = n;
    return 0;
}

int grm_engine_download(grm_engine *e, const grm_init_photon *dev, size_t n, grm_init_photon *host_out) {
    if (!e || (n && (!dev || !host_out))) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    if (n) HIPCHK(e, hipMemcpy(host_out, dev, n * sizeof(grm_init_photon), hipMemcpyDeviceToHost));
    return 0;
}

int grm_engine_debug_timing(grm_engine *e, uint64_t out[48], int reset) {
    if (!e || !out) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemcpy(out, e->d_timing, 48 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (reset) HIPCHK(e, hipMemset(e->d_timing, 0, 48 * sizeof(unsigned long long)));
#ifdef GRM_TIMING
    return 1;
#else
    return 0;
#endif
}

int64_t grm_engine_debug_waves(grm_engine *e, uint64_t *out, size_t cap) {
    if (!e || !e->d_waves) return -1;
    if (hipSetDevice(e->device) != hipSuccess) return -1;
    const size_t n = std::min(e->lanes / 64, e->waves_rows);
    const size_t k = std::min(n, cap);
    if (k && out && hipMemcpy(out, e->d_waves, k * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return (int64_t)n;
}

int grm_engine_debug_phases(grm_engine *e, uint64_t out[4]) {
    if (!e || !out) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    DevCounters h;
    if (read_counters(e, h)) return -1; /* mirrors the small words */
    unsigned long long lo = ~0ull, hi = 0;
    const size_t n = std::min(e->lanes / 64, e->waves_rows);
    if (n) {
        std::vector<unsigned long long> w(n * 4);
        HIPCHK(e, hipMemcpy(w.data(), e->d_waves, n * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; ++i) {
            lo = std::min(lo, w[i * 4]);
            hi = std::max(hi, w[i * 4 + 1]);
        }
    }
    unsigned long long ph[2] = {0, 0};
    if (n) HIPCHK(e, hipMemcpy(ph, e->d_waves + (e->lanes / 64) * 4, sizeof(ph), hipMemcpyDeviceToHost));
    out[0] = n ? lo : 0;
    out[1] = ph[0];
    out[2] = ph[1];
    out[3] = hi;
    return 0;
}

int64_t grm_engine_debug_admissions(grm_engine *e, uint64_t *out, size_t cap) {
    if (!e || !e->d_waves || !e->waves_rows) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    unsigned long long ph[PHASE_LOG];
    HIPCHK(e, hipMemcpy(ph, e->d_waves + (e->lanes / 64) * 4, sizeof(ph), hipMemcpyDeviceToHost));
    const size_t k = std::min<size_t>(ph[2], (PHASE_LOG - 3) / 2);
    for (size_t i = 0; i < k && i < cap; ++i) {
        out[2 * i] = ph[3 + 2 * i];
        out[2 * i + 1] = ph[4 + 2 * i];
    }
    return (int64_t)k;
}

int grm_engine_debug_counters(grm_engine *e, uint64_t out[16]) {
    if (!e || !out) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    DevCounters h;
    if (read_counters(e, h)) return -1;
    std::memcpy(out, &h, sizeof(h));
    return 0;
}

int64_t grm_engine_debug_stuck(grm_engine *e, double *out, size_t cap) {
    if (!e || !e->d_small) return -1;
    if (hipSetDevice(e->device) != hipSuccess) return -1;
    unsigned long long cnt = 0;
    if (hipMemcpy(&cnt, e->d_small + (6) * SMALL_STRIDE, sizeof(cnt), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    const size_t n = std::min<size_t>(cnt, STUCK_CAP), k = std::min(n, cap);
    if (k && out && hipMemcpy(out, e->d_stuck, k * STUCK_WORDS * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return (int64_t)n;
}

int grm_rccl_unique_id(uint8_t id_out[128]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

int grm_engine_comm_init(grm_engine *e, const uint8_t id_in[128], int nranks, int rank) {
    if (!e || !id_in) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    ncclUniqueId id;
    std::memcpy(&id, id_in, sizeof(id));
    const ncclResult_t r = ncclCommInitRank(&e->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        e->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        e->comm = nullptr;
        return -1;
    }
    return 0;
}

int grm_engine_allreduce(grm_engine *e) {
    if (!e) return -1;
    if (!e->comm) {
        e->err = "grm_engine_allreduce: no communicator (grm_engine_comm_init)";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    const size_t ncell = (size_t)N_TH_BINS * N_E_BINS * (sizeof(grm_spectrum_cell) / sizeof(double));
    unsigned long long *c = reinterpret_cast<unsigned long long *>(e->d_ctr);
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess) r = ncclAllReduce(e->d_spec, e->d_spec, ncell, ncclFloat64, ncclSum, e->comm, e->stream);
    /* DevCounters: [0..1] n_recorded n_scatt (sum), [2] max_tau bits (max; tau >= 0 orders as u64),
     * [3..8] steps/tracked/children/overflow/dropped/primaries (sum) */
    if (r == ncclSuccess) r = ncclAllReduce(c, c, 2, ncclUint64, ncclSum, e->comm, e->stream);
    if (r == ncclSuccess) r = ncclAllReduce(c + 2, c + 2, 1, ncclUint64, ncclMax, e->comm, e->stream);
    if (r == ncclSuccess) r = ncclAllReduce(c + 3, c + 3, 6, ncclUint64, ncclSum, e->comm, e->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess) {
        e->err = std::string("RCCL all-reduce: ") + ncclGetErrorString(r);
        return -1;
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return 0;
}

int grm_engine_stash_reserve(grm_engine *e, int n_slots) {
    if (!e || n_slots < 0) return -1;
    if (n_slots <= e->stash_cap) return 0;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const size_t ncell = (size_t)N_TH_BINS * N_E_BINS * (sizeof(grm_spectrum_cell) / sizeof(double));
    hipFree(e->d_stash_spec);
    hipFree(e->d_stash_sum);
    hipFree(e->d_stash_max);
    e->d_stash_spec = nullptr;
    e->d_stash_sum = e->d_stash_max = nullptr;
    e->stash_cap = 0;
    HIPCHK(e, hipMalloc(&e->d_stash_spec, (size_t)n_slots * ncell * sizeof(double)));
    HIPCHK(e, hipMalloc(&e->d_stash_sum, (size_t)n_slots * STASH_SUMS * sizeof(unsigned long long)));
    HIPCHK(e, hipMalloc(&e->d_stash_max, (size_t)n_slots * STASH_MAXS * sizeof(unsigned long long)));
    e->stash_cap = n_slots;
    /* per-pass counter blocks (grm_engine_begin_pass); a new allocation unlinks the peers */
    if (e->ctr_slot >= 0) e->d_ctr = e->d_ctr_own;
    e->ctr_slot = -1;
    hipFree(e->d_ctr_slots);
    e->d_ctr_slots = nullptr;
    e->n_ctr_slots = 0;
    hipFree(e->d_peers);
    e->d_peers = nullptr;
    e->n_peers = 0;
    HIPCHK(e, hipMalloc(&e->d_ctr_slots, (size_t)n_slots * sizeof(DevCounters)));
    HIPCHK(e, hipMemset(e->d_ctr_slots, 0, (size_t)n_slots * sizeof(DevCounters)));
    e->n_ctr_slots = n_slots;
    return 0;
}

int grm_engine_begin_pass(grm_engine *e, int slot) {
    if (!e) return -1;
    if (slot >= e->n_ctr_slots) {
        e->err = "grm_engine_begin_pass: slot " + std::to_string(slot) + " outside the reserved " +
                 std::to_string(e->n_ctr_slots) + " (grm_engine_stash_reserve)";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->ctr_slot = slot < 0 ? -1 : slot;
    e->d_ctr = slot < 0 ? e->d_ctr_own : e->d_ctr_slots + slot;
    return grm_engine_reset(e);
}

int grm_engine_counters_ipc_handle(grm_engine *e, uint8_t out[64]) {
    if (!e || !out) return -1;
    if (!e->d_ctr_slots) {
        e->err = "grm_engine_counters_ipc_handle: no pass slots (grm_engine_stash_reserve first)";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    hipIpcMemHandle_t h;
    HIPCHK(e, hipIpcGetMemHandle(&h, e->d_ctr_slots));
    static_assert(sizeof(h) <= 64, "IPC handle size");
    std::memset(out, 0, 64);
    std::memcpy(out, &h, sizeof(h));
    return 0;
}

namespace {
int upload_peers(grm_engine *e, const std::vector<const DevCounters *> &tab) {
    hipFree(e->d_peers);
    e->d_peers = nullptr;
    e->n_peers = 0;
    if (tab.size() < 2) return 0;
    HIPCHK(e, hipMalloc(&e->d_peers, tab.size() * sizeof(DevCounters *)));
    HIPCHK(e, hipMemcpy(e->d_peers, tab.data(), tab.size() * sizeof(DevCounters *), hipMemcpyHostToDevice));
    e->n_peers = (int)tab.size();
    return 0;
}
} /* namespace */

int grm_engine_set_peers(grm_engine *e, const uint8_t *handles, int n, int rank) {
    if (!e || n < 0 || (n > 1 && (!handles || rank < 0 || rank >= n))) return -1;
    if (n > 64) {
        e->err = "grm_engine_set_peers: at most 64 ranks";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    for (void *p : e->ipc_open) hipIpcCloseMemHandle(p);
    e->ipc_open.clear();
    std::vector<const DevCounters *> tab;
    if (n > 1) {
        if (!e->d_ctr_slots) {
            e->err = "grm_engine_set_peers: no pass slots (grm_engine_stash_reserve first)";
            return -1;
        }
        for (int r = 0; r < n; ++r) {
            if (r == rank) {
                tab.push_back(e->d_ctr_slots);
                continue;
            }
            hipIpcMemHandle_t h;
            std::memcpy(&h, handles + (size_t)r * 64, sizeof(h));
            void *p = nullptr;
            const hipError_t st = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
            if (st != hipSuccess) {
                for (void *q : e->ipc_open) hipIpcCloseMemHandle(q);
                e->ipc_open.clear();
                e->err = std::string("grm_engine_set_peers: hipIpcOpenMemHandle of rank ") + std::to_string(r) + ": " +
                         hipGetErrorString(st);
                upload_peers(e, {});
                return -1;
            }
            e->ipc_open.push_back(p);
            tab.push_back(reinterpret_cast<const DevCounters *>(p));
        }
    }
    return upload_peers(e, tab);
}

int grm_device_peer_ok(int device, int peer) {
    if (device == peer) return 1;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, device, peer) != hipSuccess) return 0;
    return can ? 1 : 0;
}

int grm_engine_link_peers(grm_engine *const *engines, int n) {
    if (!engines || n < 1) return -1;
    std::vector<const DevCounters *> tab;
    for (int r = 0; r < n; ++r) {
        if (!engines[r] || !engines[r]->d_ctr_slots || engines[r]->device != engines[0]->device) return -1;
        tab.push_back(engines[r]->d_ctr_slots);
    }
    for (int r = 0; r < n; ++r) {
        grm_engine *e = engines[r];
        HIPCHK(e, hipSetDevice(e->device));
        if (upload_peers(e, n > 1 ? tab : std::vector<const DevCounters *>{})) return -1;
    }
    return 0;
}

int grm_engine_job_counters(grm_engine *e, double out[4]) {
    if (!e || !out) return -1;
    HIPCHK(e, hipSetDevice(e->device));
    Ctl C{};
    C.ctr = e->d_ctr;
    C.peers = e->d_peers;
    C.n_peers = (e->ctr_slot >= 0 && e->d_peers) ? e->n_peers : 0;
    C.ctr_slot = e->ctr_slot;
    double *d = nullptr;
    HIPCHK(e, hipMalloc(&d, 4 * sizeof(double)));
    hipLaunchKernelGGL(job_counters_kernel, dim3(1), dim3(64), 0, e->stream, e->P, C, d);
    hipError_t st = hipGetLastError();
    if (st == hipSuccess) st = hipMemcpyAsync(out, d, 4 * sizeof(double), hipMemcpyDeviceToHost, e->stream);
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    (void)hipFree(d);
    return hip_ok(e, st, "job counters") ? 0 : -1;
}

int grm_engine_stash(grm_engine *e, int slot) {
    if (!e) return -1;
    if (slot < 0 || slot >= e->stash_cap) {
        e->err = "grm_engine_stash: slot " + std::to_string(slot) + " outside the reserved " +
                 std::to_string(e->stash_cap) + " (grm_engine_stash_reserve)";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    const int ncell = N_TH_BINS * N_E_BINS * (int)(sizeof(grm_spectrum_cell) / sizeof(double));
    hipLaunchKernelGGL(stash_kernel, dim3(8), dim3(256), 0, e->stream, reinterpret_cast<const double *>(e->d_spec),
                       e->d_ctr, e->d_stash_spec, e->d_stash_sum, e->d_stash_max, slot, ncell);
    HIPCHK(e, hipGetLastError());
    return 0;
}

int grm_engine_allreduce_stash(grm_engine *e, int first, int n_slots) {
    if (!e) return -1;
    if (first < 0 || n_slots < 0 || first + n_slots > e->stash_cap) {
        e->err = "grm_engine_allreduce_stash: slots outside the reserved stash";
        return -1;
    }
    if (!e->comm) {
        e->err = "grm_engine_allreduce_stash: no communicator (grm_engine_comm_init)";
        return -1;
    }
    if (n_slots == 0) return 0;
    HIPCHK(e, hipSetDevice(e->device));
    const size_t ncell = (size_t)N_TH_BINS * N_E_BINS * (sizeof(grm_spectrum_cell) / sizeof(double));
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess)
        r = ncclAllReduce(e->d_stash_spec + (size_t)first * ncell, e->d_stash_spec + (size_t)first * ncell,
                          (size_t)n_slots * ncell, ncclFloat64, ncclSum, e->comm, e->stream);
    if (r == ncclSuccess)
        r = ncclAllReduce(e->d_stash_sum + (size_t)first * STASH_SUMS, e->d_stash_sum + (size_t)first * STASH_SUMS,
                          (size_t)n_slots * STASH_SUMS, ncclUint64, ncclSum, e->comm, e->stream);
    if (r == ncclSuccess)
        r = ncclAllReduce(e->d_stash_max + (size_t)first * STASH_MAXS, e->d_stash_max + (size_t)first * STASH_MAXS,
                          (size_t)n_slots * STASH_MAXS, ncclUint64, ncclMax, e->comm, e->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess) {
        e->err = std::string("RCCL all-reduce (stash): ") + ncclGetErrorString(r);
        return -1;
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return 0;
}

int grm_engine_stash_read(grm_engine *e, int slot, grm_spectrum_cell *spec, uint64_t *n_rec, uint64_t *n_scatt,
                          double *max_tau, uint64_t *n_steps) {
    if (!e) return -1;
    if (slot < 0 || slot >= e->stash_cap) {
        e->err = "grm_engine_stash_read: slot outside the reserved stash";
        return -1;
    }
    HIPCHK(e, hipSetDevice(e->device));
    const size_t ncell = (size_t)N_TH_BINS * N_E_BINS * (sizeof(grm_spectrum_cell) / sizeof(double));
    unsigned long long sums[STASH_SUMS], maxs[STASH_MAXS];
    if (spec)
        HIPCHK(e, hipMemcpyAsync(spec, e->d_stash_spec + (size_t)slot * ncell, ncell * sizeof(double),
                                 hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(sums, e->d_stash_sum + (size_t)slot * STASH_SUMS, sizeof(sums), hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipMemcpyAsync(maxs, e->d_stash_max + (size_t)slot * STASH_MAXS, sizeof(maxs), hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (n_rec) *n_rec = sums[0];
    if (n_scatt) *n_scatt = sums[1];
    if (n_steps) *n_steps = sums[2];
    if (max_tau) std::memcpy(max_tau, &maxs[0], sizeof(double));
    return 0;
}

int grm_engine_stash_raw(grm_engine *e, int first, int n_slots, double *spec, uint64_t *sums, uint64_t *maxs,
                         int write) {
    if (!e) return -1;
    if (first < 0 || n_slots < 0 || first + n_slots > e->stash_cap) {
        e->err = "grm_engine_stash_raw: slots outside the reserved stash";
        return -1;
    }
    if (n_slots == 0) return 0;
    HIPCHK(e, hipSetDevice(e->device));
    const size_t ncell = (size_t)N_TH_BINS * N_E_BINS * (sizeof(grm_spectrum_cell) / sizeof(double));
    const hipMemcpyKind k = write ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
    struct Part {
        void *dev, *host;
        size_t bytes;
    } parts[3] = {{e->d_stash_spec + (size_t)first * ncell, spec, (size_t)n_slots * ncell * sizeof(double)},
                  {e->d_stash_sum + (size_t)first * STASH_SUMS, sums, (size_t)n_slots * STASH_SUMS * sizeof(uint64_t)},
                  {e->d_stash_max + (size_t)first * STASH_MAXS, maxs, (size_t)n_slots * STASH_MAXS * sizeof(uint64_t)}};
    for (const Part &q : parts) {
        if (!q.host) continue;
        if (write)
            HIPCHK(e, hipMemcpyAsync(q.dev, q.host, q.bytes, k, e->stream));
        else
            HIPCHK(e, hipMemcpyAsync(q.host, q.dev, q.bytes, k, e->stream));
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return 0;
}

int grm_stash_words(int which) {
    switch (which) {
    case 0: return N_TH_BINS * N_E_BINS * (int)(sizeof(grm_spectrum_cell) / sizeof(double));
    case 1: return STASH_SUMS;
    case 2: return STASH_MAXS;
    default: return -1;
    }
}

int grm_probe(grm_engine *e, int which, const double *in, int in_stride, double *out, int out_stride, size_t n) {
    if (!e) return -1;
    hipSetDevice(e->device);
    return grm_probe_impl(e->P, e->stream, which, in, in_stride, out, out_stride, n, e->err);
}

size_t grm_sizeof(int which) {
    switch (which) {
    case 0: return sizeof(grm_header);
    case 1: return sizeof(grm_units);
    case 2: return sizeof(grm_init_photon);
    case 3: return sizeof(grm_spectrum_cell);
    case 4: return sizeof(grm_trace);
    case 5: return sizeof(grm_stats);
    case 6: return sizeof(grm_emit_zone);
    default: return 0;
    }
}

const char *grm_version(void) { return "grmonty_amd 0.1.0 (gfx950)"; }

} /* extern "C" */
#endif /* !GRM_LONE_TU && !GRM_SPLIT_TU */
