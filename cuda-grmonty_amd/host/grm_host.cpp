/*
 * grm_host.cpp -- C++ host side of the engine: HARM dump loader, units, init tables,
 * zone-parallel superphoton emission, spectrum writer (include/grmonty_amd.h, "host model").
 *
 * Reference counterparts (m-torhan/cuda-grmonty):
 *   HARMModel::HARMModel / read_file        harm_model.cpp:64-232
 *   init_geometry / init_weight_table /
 *   init_nint_table                         harm_model.cpp:242-338
 *   hotcross::init_table                    hotcross.cpp:60-79 (+ :108-181)
 *   jnu_mixed::init_emiss_tables            jnu_mixed.cpp:57-73 (+ integration.cpp GK61)
 *   get_zone / init_zone / sample_zone_photon /
 *   make_super_photon(_async)               harm_model.cpp:673-892, 1337-1389
 *   report_spectrum                         harm_model.cpp:416-471
 *
 * Differences by design (MI355X host):
 *   - tables are built multi-threaded; every table entry is computed with the reference's
 *     arithmetic in the reference's summation order, so they are bit-identical to a serial
 *     build (tests/test_tables.py checks against the oracle);
 *   - emission is zone-parallel and deterministic: zone z draws from its own Philox4x32-10
 *     stream (key = seed, counter = (draw, zone, salt)), so the emitted photon list depends
 *     only on the seed, never on the thread count.  The reference's CUDA build instead feeds
 *     4 mt19937 worker threads from a zone master (harm_model.cpp:813-892; its output depends
 *     on thread timing).
 */
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <queue>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/grmonty_amd.h"

namespace {

/* ---- constants (consts.hpp:14-157) ---- */
constexpr double kPi = 3.141592653589793238462643383279502884;
constexpr double kSqrt2 = 1.414213562373095048801688724209698079;
constexpr double kLn10 = 2.302585092994045684017991454684364208;
constexpr double EPS = 1.0e-40;
constexpr int NSAMP = GRM_N_E_SAMP;
constexpr double NU_MIN = 1.0e9, NU_MAX = 1.0e16;
constexpr double THETA_E_MIN = 0.3, TP_OVER_TE = 3.0;
constexpr double EE = 4.80320680e-10, CL = 2.99792458e10, ME = 9.1093826e-28, MP = 1.67262171e-24;
constexpr double HPL = 6.6260693e-27, HBAR = HPL / (2. * kPi), G_NEWT = 6.6742e-8;
constexpr double SIGMA_THOMSON = 0.665245873e-24;
constexpr double M_SUN = 1.989e33, L_SUN = 3.827e33, M_BH = 4.0e6 * M_SUN;
constexpr int NINT = GRM_NINT;
constexpr double BTHSQ_MIN = 1.0e-4, BTHSQ_MAX = 1.0e8;
constexpr double HC_MIN_W = 1.0e-12, HC_MAX_W = 1.0e6, HC_MIN_T = 1.0e-4, HC_MAX_T = 1.0e4;
constexpr int HC_N_W = GRM_HC_N_W, HC_N_T = GRM_HC_N_T;
constexpr double HC_MAX_GAMMA = 12.0, HC_D_MU_E = 0.05, HC_D_GAMMA_E = 0.05;
constexpr double JNU_MIN_K = 0.002, JNU_MAX_K = 1.0e7, JNU_MAX_T = 1.0e2;
constexpr double JNU_CST = 1.88774862536;
constexpr double JNU_K_FAC = 9 * kPi * ME * CL / EE;
constexpr double JCST = kSqrt2 * EE * EE * EE / (27.0 * ME * CL * CL);
constexpr double SPEC_D_L_E = 0.25;

struct Consts {
    double l_nu_min, n_l_n, d_l_nu, l_b_min, d_l_b;
    double hc_l_min_w, hc_l_min_t, hc_d_l_w, hc_d_l_t;
    double jnu_l_min_k, jnu_d_l_k, jnu_l_min_t, jnu_d_l_t, spec_l_e_0;
    Consts() {
        l_nu_min = std::log(NU_MIN);
        const double l_nu_max = std::log(NU_MAX);
        n_l_n = l_nu_max - l_nu_min;
        d_l_nu = (l_nu_max - l_nu_min) / NSAMP;
        l_b_min = std::log(BTHSQ_MIN);
        d_l_b = std::log(BTHSQ_MAX / BTHSQ_MIN) / NINT;
        hc_l_min_w = std::log10(HC_MIN_W);
        hc_l_min_t = std::log10(HC_MIN_T);
        hc_d_l_w = std::log10(HC_MAX_W / HC_MIN_W) / HC_N_W;
        hc_d_l_t = std::log10(HC_MAX_T / HC_MIN_T) / HC_N_T;
        jnu_l_min_k = std::log(JNU_MIN_K);
        jnu_d_l_k = std::log(JNU_MAX_K / JNU_MIN_K) / NSAMP;
        jnu_l_min_t = std::log(THETA_E_MIN);
        jnu_d_l_t = std::log(JNU_MAX_T / THETA_E_MIN) / NSAMP;
        spec_l_e_0 = std::log(1.0e-12);
    }
};
const Consts K;

thread_local std::string g_err;

/* ---- Philox4x32-10 (host copy of the device stream definition) ---- */
struct Philox {
    uint32_t k0, k1, c2, c3;
    uint64_t ctr = 0;
    double uniform() {
        uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), a2 = c2, a3 = c3, q0 = k0, q1 = k1;
        for (int r = 0; r < 10; ++r) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * a2;
            const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ q0;
            const uint32_t n2 = (uint32_t)(p0 >> 32) ^ a3 ^ q1;
            c0 = n0;
            c1 = (uint32_t)p1;
            a2 = n2;
            a3 = (uint32_t)p0;
            q0 += 0x9E3779B9u;
            q1 += 0xBB67AE85u;
        }
        ++ctr;
        const uint64_t m = ((((uint64_t)c1) << 32) | c0) >> 11;
        return (double)(m + 1) * (1.0 / 9007199254740992.0);
    }
};

/* emission streams of zone z: counter words 2,3 = (zone, salt 'EMIT'), word 1 = slot (0 = the
 * zone's count draw, p + 1 = photon p of the zone), word 0 = draw index.  Photons of one zone are
 * independent streams, so any lane / thread can sample any photon (the device emitter does). */
Philox zone_stream(uint64_t seed, uint64_t zone, uint64_t slot = 0) {
    Philox p;
    p.k0 = (uint32_t)seed;
    p.k1 = (uint32_t)(seed >> 32);
    p.c2 = (uint32_t)zone;
    p.c3 = 0x454D4954u ^ (uint32_t)(zone >> 32);
    p.ctr = slot << 32;
    return p;
}

/* ---- GK61 (integration.cpp:144-236), QUADPACK 61-point Kronrod rule ---- */
const double XK[31] = {
    0.999484410050490637571325895705811, 0.996893484074649540271630050918695, 0.991630996870404594858628366109486,
    0.983668123279747209970032581605663, 0.973116322501126268374693868423707, 0.960021864968307512216871025581798,
    0.944374444748559979415831324037439, 0.926200047429274325879324277080474, 0.905573307699907798546522558925958,
    0.882560535792052681543116462530226, 0.857205233546061098958658510658944, 0.829565762382768397442898119732502,
    0.799727835821839083013668942322683, 0.767777432104826194917977340974503, 0.733790062453226804726171131369528,
    0.697850494793315796932292388026640, 0.660061064126626961370053668149271, 0.620526182989242861140477556431189,
    0.579345235826361691756024932172540, 0.536624148142019899264169793311073, 0.492480467861778574993693061207709,
    0.447033769538089176780609900322854, 0.400401254830394392535476211542661, 0.352704725530878113471037207089374,
    0.304073202273625077372677107199257, 0.254636926167889846439805129817805, 0.204525116682309891438957671002025,
    0.153869913608583546963794672743256, 0.102806937966737030147096751318001, 0.051471842555317695833025213166723,
    0.0};
const double WK[31] = {
    0.001389013698677007624551591226760, 0.003890461127099884051267201844516, 0.006630703915931292173319826369750,
    0.009273279659517763428441146892024, 0.011823015253496341742232898853251, 0.014369729507045804812451432443580,
    0.016920889189053272627572289420322, 0.019414141193942381173408951050128, 0.021828035821609192297167485738339,
    0.024191162078080601365686370725232, 0.026509954882333101610601709335075, 0.028754048765041292843978785354334,
    0.030907257562387762472884252943092, 0.032981447057483726031814191016854, 0.034979338028060024137499670731468,
    0.036882364651821229223911065617136, 0.038678945624727592950348651532281, 0.040374538951535959111995279752468,
    0.041969810215164246147147541285970, 0.043452539701356069316831728117073, 0.044814800133162663192355551616723,
    0.046059238271006988116271735559374, 0.047185546569299153945261478181099, 0.048185861757087129140779492298305,
    0.049055434555029778887528165367238, 0.049795683427074206357811569379942, 0.050405921402782346840893085653585,
    0.050881795898749606492297473049805, 0.051221547849258772170656282604944, 0.051426128537459025933862879215781,
    0.051494729429451567558340433647099};
const double WG[15] = {
    0.007968192496166605615465883474674, 0.018466468311090959142302131912047, 0.028784707883323369349719179611292,
    0.038799192569627049596801936446348, 0.048402672830594052902938140422808, 0.057493156217619066481721689402056,
    0.065974229882180495128128515115962, 0.073755974737705206268243850022191, 0.080755895229420215354694938460530,
    0.086899787201082979802387530715126, 0.092122522237786128717632707087619, 0.096368737174644259639468626351810,
    0.099593420586795267062780282103569, 0.101762389748405504596428952168554, 0.102852652893558840341285636705415};

struct Piece {
    double a, b, val, err;
    bool operator<(const Piece &o) const { return err < o.err; }
};

Piece kronrod61(const std::function<double(double)> &f, double a, double b) {
    const double c = 0.5 * (a + b), h = 0.5 * (b - a);
    double fv1[30], fv2[30];
    const double fc = f(c);
    double rk = fc * WK[30], rg = 0.0, rabs = std::abs(fc) * WK[30];
    for (int i = 0; i < 30; ++i) {
        const double d = h * XK[i];
        fv1[i] = f(c - d);
        fv2[i] = f(c + d);
        const double s = fv1[i] + fv2[i];
        rk += WK[i] * s;
        rabs += WK[i] * (std::abs(fv1[i]) + std::abs(fv2[i]));
        if (i & 1) rg += WG[i >> 1] * s;
    }
    rk *= h;
    rg *= h;
    rabs *= h;
    const double mean = rk / (b - a);
    double rasc = WK[30] * std::abs(fc - mean);
    for (int i = 0; i < 30; ++i) rasc += WK[i] * (std::abs(fv1[i] - mean) + std::abs(fv2[i] - mean));
    rasc *= h;
    double err = std::abs(rk - rg);
    if (rasc != 0.0 && err != 0.0) {
        const double sc = std::pow(200.0 * err / rasc, 1.5);
        err = sc < 1.0 ? rasc * sc : rasc;
    }
    if (rasc == 0.0 || err < 50 * std::numeric_limits<double>::epsilon() * rabs) err = 0.0;
    return {a, b, rk, err};
}

double adaptive_gk61(const std::function<double(double)> &f, double a, double b, double eps_abs, double eps_rel,
                     int max_pieces) {
    std::priority_queue<Piece> heap;
    Piece p0 = kronrod61(f, a, b);
    heap.push(p0);
    double total = p0.val, total_err = p0.err;
    int used = 1;
    while (!heap.empty() && total_err > std::max(eps_abs, eps_rel * std::abs(total))) {
        if (used >= max_pieces) throw std::runtime_error("GK61 did not converge");
        const Piece cur = heap.top();
        heap.pop();
        const double mid = 0.5 * (cur.a + cur.b);
        const Piece l = kronrod61(f, cur.a, mid), r = kronrod61(f, mid, cur.b);
        total += (l.val + r.val - cur.val);
        total_err += (l.err + r.err - cur.err);
        heap.push(l);
        heap.push(r);
        ++used;
    }
    return total;
}

double klein_nishina_sigma(double w) { /* hotcross.cpp:144-151 */
    if (w < 1.0e-3) return (1.0 - 2.0 * w);
    return (3.0 / 4.0) * (2.0 / (w * w) + (1.0 / (2.0 * w) - (1.0 + w) / (w * w * w)) * std::log(1.0 + 2.0 * w) +
                          (1.0 + w) / ((1.0 + 2.0 * w) * (1.0 + 2.0 * w)));
}

/* hot cross section by quadrature over electron angle/energy (hotcross.cpp:108-142).  The
 * Maxwell-Juttner weight depends on (theta_e, gamma_e) only: computed once per column. */
struct HotColumn {
    std::vector<double> gam, fw, v;
};

HotColumn hot_column(double theta_e) {
    HotColumn c;
    const double k2f = theta_e > 1.0e-2 ? std::cyl_bessel_k(2, 1.0 / theta_e) * std::exp(1.0 / theta_e)
                                        : std::sqrt(kPi * theta_e / 2.0);
    for (double g = 1.0 + 0.5 * theta_e * HC_D_GAMMA_E; g < 1.0 + HC_MAX_GAMMA * theta_e; g += theta_e * HC_D_GAMMA_E) {
        c.gam.push_back(g);
        c.fw.push_back(0.5 * ((g * std::sqrt(g * g - 1.) / (theta_e * k2f)) * std::exp(-(g - 1.) / theta_e)));
        c.v.push_back(std::sqrt(g * g - 1.0) / g);
    }
    return c;
}

double hot_sigma(double w, double theta_e, const HotColumn &c) {
    if (std::isnan(w)) return 0.0;
    if (theta_e < HC_MIN_T && w < HC_MIN_W) return SIGMA_THOMSON;
    if (theta_e < HC_MIN_T) return klein_nishina_sigma(w) * SIGMA_THOMSON;
    double cross = 0.0;
    for (double mu = -1.0 + 0.5 * HC_D_MU_E; mu < 1.0; mu += HC_D_MU_E)
        for (size_t t = 0; t < c.gam.size(); ++t) {
            const double f = 1.0 - mu * c.v[t];
            cross += theta_e * HC_D_MU_E * HC_D_GAMMA_E * (klein_nishina_sigma(w * c.gam[t] * f) * f) * c.fw[t];
        }
    return cross * SIGMA_THOMSON;
}

/* default worker count: OMP_NUM_THREADS if set, else min(16, cores) -- a GPU box reports the
 * whole machine's CPUs but one GPU's share is 16 */
int default_threads() {
    if (const char *v = std::getenv("OMP_NUM_THREADS")) {
        const int n = std::atoi(v);
        if (n > 0) return n;
    }
    return (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
}

void parallel_for(int n, int n_threads, const std::function<void(int)> &body) {
    if (n_threads < 1) n_threads = default_threads();
    n_threads = std::min(n_threads, std::max(n, 1));
    std::atomic<int> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t)
        th.emplace_back([&]() {
            for (int i = next++; i < n; i = next++) body(i);
        });
    for (auto &t : th) t.join();
}

struct Fluid {
    double n_e, theta_e, b;
    double u_con[4], b_con[4];
};

} /* namespace */

struct grm_model {
    grm_header hdr{};
    grm_units units{};
    int photon_n = 0;
    std::vector<double> fld[8];
    double bias_norm = 0, rh = 0, x1_min = 0, max_tau_scatt = 0, d_tau_k = 0;
    std::vector<double> hot, k2, ftab, weight, nint, dndlnu_max;
    double table_ms = 0.0; /* GPU time of the device table builders (grm_model_init_device) */
    std::vector<double> gcov, gcon0, det; /* per zone: 16, 4 (row 0 of g^mu nu), 1 */
    bool inited = false;
    int n1() const { return hdr.n[0]; }
    int n2() const { return hdr.n[1]; }
    double F(int f, int i, int j) const { return fld[f][(size_t)i * hdr.n[1] + j]; }
};

namespace {

void bl(const grm_model *m, const double x[4], double &r, double &th) { /* harm_model.cpp:1632-1637 */
    r = std::exp(x[1]) + m->hdr.r_0;
    th = kPi * x[2] + ((1.0 - m->hdr.h_slope) / 2.0) * std::sin(2.0 * kPi * x[2]);
}

void metric_cov(const grm_model *m, const double x[4], double g[16]) { /* :499-530 */
    double r, th;
    bl(m, x, r, th);
    const double a = m->hdr.a;
    const double st = std::fabs(std::sin(th)) + EPS, ct = std::cos(th);
    const double s2 = st * st, rho2 = r * r + a * a * ct * ct, rfac = r - m->hdr.r_0;
    const double hfac = kPi + (1.0 - m->hdr.h_slope) * kPi * std::cos(2.0 * kPi * x[2]);
    std::fill(g, g + 16, 0.0);
    g[0] = (-1.0 + 2.0 * r / rho2);
    g[1] = g[4] = (2.0 * r / rho2) * rfac;
    g[3] = g[12] = (-2.0 * a * r * s2 / rho2);
    g[5] = (1.0 + 2.0 * r / rho2) * rfac * rfac;
    g[7] = g[13] = (-a * s2 * (1.0 + 2.0 * r / rho2)) * rfac;
    g[10] = rho2 * hfac * hfac;
    g[15] = s2 * (rho2 + a * a * s2 * (1.0 + 2.0 * r / rho2));
}

void metric_con_row0(const grm_model *m, const double x[4], double g0[4]) { /* :473-497, row 0 */
    double r, th;
    bl(m, x, r, th);
    const double a = m->hdr.a, ct = std::cos(th);
    const double irho2 = 1.0 / (r * r + a * a * ct * ct);
    g0[0] = -1.0 - 2.0 * r * irho2;
    g0[1] = 2.0 * irho2;
    g0[2] = 0.0;
    g0[3] = 0.0;
}

double det4(const double *a) {
    auto m3 = [&](int c0, int c1, int c2) {
        return a[4 + c0] * (a[8 + c1] * a[12 + c2] - a[8 + c2] * a[12 + c1]) -
               a[4 + c1] * (a[8 + c0] * a[12 + c2] - a[8 + c2] * a[12 + c0]) +
               a[4 + c2] * (a[8 + c0] * a[12 + c1] - a[8 + c1] * a[12 + c0]);
    };
    return a[0] * m3(1, 2, 3) - a[1] * m3(0, 2, 3) + a[2] * m3(0, 1, 3) - a[3] * m3(0, 1, 2);
}

void zone_coord(const grm_model *m, int i, int j, double x[4]) { /* :1639-1644 */
    x[0] = m->hdr.x_start[0];
    x[1] = m->hdr.x_start[1] + (i + 0.5) * m->hdr.dx[1];
    x[2] = m->hdr.x_start[2] + (j + 0.5) * m->hdr.dx[2];
    x[3] = m->hdr.x_start[3];
}

void lower4(const double u[4], const double *g, double uc[4]) {
    for (int i = 0; i < 4; ++i) uc[i] = g[i * 4 + 0] * u[0] + g[i * 4 + 1] * u[1] + g[i * 4 + 2] * u[2] + g[i * 4 + 3] * u[3];
}

Fluid zone_fluid(const grm_model *m, int i, int j) { /* get_fluid_zone, harm_model.cpp:538-593 */
    Fluid r{};
    const size_t z = (size_t)i * m->n2() + j;
    const double *gc = &m->gcov[z * 16];
    const double *g0 = &m->gcon0[z * 4];
    const double vc[4] = {0.0, m->F(2, i, j), m->F(3, i, j), m->F(4, i, j)};
    const double b[4] = {0.0, m->F(5, i, j), m->F(6, i, j), m->F(7, i, j)};
    r.n_e = m->F(0, i, j) * m->units.n_e_unit;
    r.theta_e = (m->F(1, i, j) / r.n_e) * m->units.n_e_unit * m->units.theta_e_unit;
    double vdv = 0.0;
    for (int a = 1; a < 4; ++a)
        for (int c = 1; c < 4; ++c) vdv += gc[a * 4 + c] * vc[a] * vc[c];
    const double vfac = std::sqrt(-1.0 / g0[0] * (1.0 + std::abs(vdv)));
    r.u_con[0] = -vfac * g0[0];
    for (int a = 1; a < 4; ++a) r.u_con[a] = vc[a] - vfac * g0[a];
    double uc[4], bc[4];
    lower4(r.u_con, gc, uc);
    double udb = 0.0;
    for (int a = 1; a < 4; ++a) udb += uc[a] * b[a];
    r.b_con[0] = udb;
    for (int a = 1; a < 4; ++a) r.b_con[a] = (b[a] + r.u_con[a] * udb) / r.u_con[0];
    lower4(r.b_con, gc, bc);
    r.b = std::sqrt(r.b_con[0] * bc[0] + r.b_con[1] * bc[1] + r.b_con[2] * bc[2] + r.b_con[3] * bc[3]) *
          m->units.b_unit;
    return r;
}

double k2_eval(const grm_model *m, double theta_e) { /* jnu_mixed.cpp:102-111, 150-158 */
    if (theta_e < THETA_E_MIN) return 0.0;
    if (theta_e > JNU_MAX_T) return 2.0 * theta_e * theta_e;
    double d = (std::log(theta_e) - K.jnu_l_min_t) / K.jnu_d_l_t;
    const int i = std::min((int)d, NSAMP - 1);
    d -= i;
    return std::exp((1.0 - d) * m->k2[i] + d * m->k2[i + 1]);
}

double f_eval(const grm_model *m, double theta_e, double b_mag, double nu) { /* jnu_mixed.cpp:113-125 */
    const double k = JNU_K_FAC * nu / (b_mag * theta_e * theta_e);
    if (k > JNU_MAX_K) return 0.0;
    if (k < JNU_MIN_K) {
        const double x = std::pow(k, 1.0 / 3.0);
        return x * (37.67503800178 + 2.240274341836 * x);
    }
    double d = (std::log(k) - K.jnu_l_min_k) / K.jnu_d_l_k;
    const int i = std::min((int)d, NSAMP - 1);
    d -= i;
    return std::exp((1.0 - d) * m->ftab[i] + d * m->ftab[i + 1]);
}

double synch(const grm_model *m, double nu, double n_e, double theta_e, double b, double theta) {
    if (theta_e < THETA_E_MIN) return 0.0; /* jnu_mixed.cpp:75-100 */
    const double k2 = k2_eval(m, theta_e);
    const double nu_c = EE * b / (2.0 * kPi * ME * CL);
    const double nu_s = (2.0 / 9.0) * nu_c * theta_e * theta_e * std::sin(theta);
    if (nu > 1.0e12 * nu_s) return 0.0;
    const double x = nu / nu_s;
    const double xp = std::pow(x, 1.0 / 3.0);
    const double xx = std::sqrt(x) + JNU_CST * std::sqrt(xp);
    return (kSqrt2 * kPi * EE * EE * n_e * nu_s / (3.0 * CL * k2)) * (xx * xx) * std::exp(-xp);
}

/* make_tetrad (tetrads.cpp:68-124) on a full 4x4 g_cov */
double gd(const double *g, const double *a, const double *b) {
    double s = 0.0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += a[i] * b[j] * g[i * 4 + j];
    return s;
}
void nrm(double *v, const double *g) {
    const double n = std::sqrt(std::abs(gd(g, v, v)));
    for (int i = 0; i < 4; ++i) v[i] /= n;
}
void proj(double *a, const double *b, const double *g) {
    const double bb = gd(g, b, b), ab = gd(g, a, b);
    for (int i = 0; i < 4; ++i) a[i] -= b[i] * ab / bb;
}
void tetrad(const double u[4], double tr[4], const double *g, double ec[4][4], double el[4][4]) {
    for (int i = 0; i < 4; ++i) ec[0][i] = u[i];
    nrm(ec[0], g);
    if (gd(g, tr, tr) < 1.0e-30)
        for (int i = 0; i < 4; ++i) tr[i] = (i == 1);
    for (int i = 0; i < 4; ++i) ec[1][i] = tr[i];
    proj(ec[1], ec[0], g);
    nrm(ec[1], g);
    for (int i = 0; i < 4; ++i) ec[2][i] = (i == 2);
    proj(ec[2], ec[0], g);
    proj(ec[2], ec[1], g);
    nrm(ec[2], g);
    for (int i = 0; i < 4; ++i) ec[3][i] = (i == 3);
    proj(ec[3], ec[0], g);
    proj(ec[3], ec[1], g);
    proj(ec[3], ec[2], g);
    nrm(ec[3], g);
    for (int i = 0; i < 4; ++i) lower4(ec[i], g, el[i]);
    for (int i = 0; i < 4; ++i) el[0][i] *= -1.0;
}

/* init_zone (harm_model.cpp:1337-1389): expected photon count and dn_max of zone (i,j) */
void zone_budget(const grm_model *m, int i, int j, double &nz, double &dn_max) {
    nz = dn_max = 0.0;
    const Fluid fz = zone_fluid(m, i, j);
    if (fz.n_e == 0.0 || fz.theta_e < THETA_E_MIN) return;
    double d_l = (std::log(fz.b * fz.theta_e * fz.theta_e) - K.l_b_min) / (K.d_l_b);
    const int l = (int)d_l;
    d_l -= l;
    if (l < 0) return;
    double ninterp = 0.0, dmax = 0.0;
    if (l >= NINT) {
        for (int q = 0; q <= NSAMP; ++q) {
            /* reference quirk kept: the frequency uses the zone's x2 index (harm_model.cpp:1362) */
            const double dn = f_eval(m, fz.theta_e, fz.b, std::exp(j * K.d_l_nu + K.l_nu_min)) /
                              (std::exp(m->weight[q]) + 1.0e-100);
            if (dn > dmax) dmax = dn;
            ninterp += K.d_l_nu * dn;
        }
    } else if (!std::isinf(m->nint[l]) && !std::isinf(m->nint[l + 1])) {
        ninterp = std::exp((1.0 - d_l) * m->nint[l] + d_l * m->nint[l + 1]);
        dmax = std::exp((1.0 - d_l) * m->dndlnu_max[l] + d_l * m->dndlnu_max[l + 1]);
    }
    const double k2 = k2_eval(m, fz.theta_e);
    if (k2 == 0.0) return;
    const double n = m->det[(size_t)i * m->n2() + j] * fz.n_e * fz.b * fz.theta_e * fz.theta_e * ninterp / k2;
    if (n > m->photon_n * std::log(NU_MAX / NU_MIN)) return;
    nz = n;
    dn_max = dmax;
}

double interp_weight(const grm_model *m, double nu) { /* :784-792 */
    double d = (std::log(nu) - K.l_nu_min) / K.d_l_nu;
    const int i = std::min((int)d, NSAMP - 1); /* u = 1 exactly -> nu = nu_max */
    d -= i;
    return std::exp((1.0 - d) * m->weight[i] + d * m->weight[i + 1]);
}

/* zone's photon count: stochastic rounding with the zone stream's first draw (:693-697) */
int zone_count(const grm_model *m, uint64_t seed, int i, int j) {
    double nz, dn_max;
    zone_budget(m, i, j, nz, dn_max);
    Philox rs = zone_stream(seed, (uint64_t)i * m->n2() + j);
    return (std::fmod(nz, 1.0) > rs.uniform()) ? (int)nz + 1 : (int)nz;
}

/* emission record of zone (i,j): init_zone (:1337-1389), the zone centre, get_fluid_zone and the
 * fluid-frame tetrad that sample_zone_photon builds for a zone's first photon (:717-731) */
void zone_record(const grm_model *m, int i, int j, grm_emit_zone &r) {
    std::memset(&r, 0, sizeof(r));
    zone_budget(m, i, j, r.nz, r.dn_max);
    zone_coord(m, i, j, r.x);
    if (!(r.nz > 0.0)) return; /* count is 0 for every seed */
    const Fluid fz = zone_fluid(m, i, j);
    r.n_e = fz.n_e;
    r.theta_e = fz.theta_e;
    r.b = fz.b;
    double bh[4];
    if (fz.b > 0.0) {
        for (int q = 0; q < 4; ++q) bh[q] = fz.b_con[q] * m->units.b_unit / fz.b;
    } else {
        bh[1] = bh[2] = bh[3] = 0.0;
        bh[0] = 1.0;
    }
    double ec[4][4], el[4][4];
    tetrad(fz.u_con, bh, &m->gcov[((size_t)i * m->n2() + j) * 16], ec, el);
    for (int a = 0; a < 4; ++a) {
        for (int b = 0; b < 4; ++b) r.e_con[a][b] = ec[a][b];
        r.e_cov_t[a] = el[a][0];
        r.e_cov_z[a] = el[a][3];
    }
}

/* sample_zone_photon (harm_model.cpp:706-782) for photons [0, count) of zone z, photon p from
 * stream slot p + 1 */
void emit_zone(const grm_model *m, const grm_emit_zone &r, uint64_t seed, uint64_t z, int count,
               grm_init_photon *out) {
    for (int p = 0; p < count; ++p) {
        Philox rs = zone_stream(seed, z, (uint64_t)p + 1);
        grm_init_photon &ph = out[p];
        std::memset(&ph, 0, sizeof(ph));
        for (int q = 0; q < 4; ++q) ph.x[q] = r.x[q];
        double nu, w;
        do {
            nu = std::exp(rs.uniform() * K.n_l_n + K.l_nu_min);
            w = interp_weight(m, nu);
        } while (rs.uniform() > (f_eval(m, r.theta_e, r.b, nu) / (w + 1.0e-100)) / r.dn_max);
        ph.w = w;
        const double j_max = synch(m, nu, r.n_e, r.theta_e, r.b, kPi / 2.0);
        double cos_th, th;
        do {
            cos_th = 2.0 * rs.uniform() - 1.0;
            th = std::acos(cos_th);
        } while (rs.uniform() > (synch(m, nu, r.n_e, r.theta_e, r.b, th) / j_max));
        const double sin_th = std::sqrt(1.0 - cos_th * cos_th);
        const double phi = 2.0 * kPi * rs.uniform();
        const double e = nu * HPL / (ME * CL * CL);
        double kt[4] = {e, e * cos_th, e * sin_th * std::cos(phi), e * sin_th * std::sin(phi)};
        for (int a = 0; a < 4; ++a) {
            ph.k[a] = 0.0;
            for (int b = 0; b < 4; ++b) ph.k[a] += r.e_con[b][a] * kt[b];
        }
        kt[0] *= -1.0;
        double t0 = 0.0, t3 = 0.0;
        for (int b = 0; b < 4; ++b) {
            t0 += r.e_cov_t[b] * kt[b];
            t3 += r.e_cov_z[b] * kt[b];
        }
        ph.e = -t0;
        ph.e_0 = -t0;
        ph.l = t3;
        ph.n_e_0 = r.n_e;
        ph.theta_e_0 = r.theta_e;
        ph.b_0 = r.b;
        ph.n_scatt = 0;
    }
}

int set_err(const std::string &s) {
    g_err = s;
    return -1;
}

/* fast whitespace tokenizer over the whole file */
struct Tok {
    const char *p, *e;
    bool next(double &v) {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p;
        if (p >= e) return false;
        char *end;
        v = std::strtod(p, &end);
        if (end == p) return false;
        p = end;
        return true;
    }
};

} /* namespace */

extern "C" {

const char *grm_model_last_error(void) { return g_err.c_str(); }

/* HARMModel(photon_n, mass_unit) + read_file (harm_model.cpp:64-232) */
int grm_model_load(const char *path, int photon_n, double mass_unit, grm_model **out) {
    if (!path || !out) return set_err("null argument");
    *out = nullptr;
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return set_err(std::string("File does not exist ") + path);
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    std::vector<char> buf((size_t)std::max(sz, 0L) + 1);
    const size_t got = std::fread(buf.data(), 1, (size_t)std::max(sz, 0L), fp);
    std::fclose(fp);
    buf[got] = 0;
    Tok t{buf.data(), buf.data() + got};
    grm_model *m = new grm_model();
    m->photon_n = photon_n;
    grm_units &u = m->units;
    u.mass_unit = mass_unit;
    u.l_unit = G_NEWT * M_BH / (CL * CL);
    u.t_unit = u.l_unit / CL;
    u.rho_unit = u.mass_unit / std::pow(u.l_unit, 3);
    u.u_unit = u.rho_unit * CL * CL;
    u.b_unit = CL * std::sqrt(4.0 * kPi * u.rho_unit);
    u.n_e_unit = u.rho_unit / (MP + ME);
    m->max_tau_scatt = 6.0 * u.l_unit * u.rho_unit * 0.4;
    m->d_tau_k = 2.0 * kPi * u.l_unit / (ME * CL * CL / HBAR);
    grm_header &h = m->hdr;
    double v[26];
    for (int q = 0; q < 26; ++q)
        if (!t.next(v[q])) {
            delete m;
            return set_err("truncated HARM header");
        }
    h.t = v[0];
    h.n[0] = (int)v[1];
    h.n[1] = (int)v[2];
    h.x_start[0] = 0.0;
    h.x_start[1] = v[3];
    h.x_start[2] = v[4];
    h.x_start[3] = 0.0;
    h.dx[0] = 1.0;
    h.dx[1] = v[5];
    h.dx[2] = v[6];
    h.dx[3] = 2.0 * kPi;
    h.x_stop[0] = 1.0;
    h.x_stop[1] = h.x_start[1] + h.n[0] * h.dx[1];
    h.x_stop[2] = h.x_start[2] + h.n[1] * h.dx[2];
    h.x_stop[3] = 2.0 * kPi;
    h.t_final = v[7];
    h.n_step = (int)v[8];
    h.a = v[9];
    h.gamma = v[10];
    h.courant = v[11];
    h.dt_dump = v[12];
    h.dt_log = v[13];
    h.dt_img = v[14];
    h.dt_rdump = (int)v[15];
    h.cnt_dump = (int)v[16];
    h.cnt_img = (int)v[17];
    h.cnt_rdump = (int)v[18];
    h.dt = v[19];
    h.lim = (int)v[20];
    h.failed = (int)v[21];
    h.r_in = v[22];
    h.r_out = v[23];
    h.h_slope = v[24];
    h.r_0 = v[25];
    if (h.n[0] < 1 || h.n[1] < 1) {
        delete m;
        return set_err("bad grid size in HARM header");
    }
    const double ttg = 0.5 * ((1. + 2. / 3. * (TP_OVER_TE + 1.) / (TP_OVER_TE + 2.)) + h.gamma);
    u.theta_e_unit = (ttg - 1.) * (MP / ME) / (1. + TP_OVER_TE);
    const size_t nz = (size_t)h.n[0] * h.n[1];
    for (auto &f : m->fld) f.assign(nz, 0.0);
    const double d_v = h.dx[1] * h.dx[2] * h.dx[3];
    double vol = 0.0, bn = 0.0;
    for (size_t z = 0; z < nz; ++z) {
        double tok[34];
        for (int q = 0; q < 34; ++q)
            if (!t.next(tok[q])) {
                delete m;
                return set_err("truncated HARM data at zone " + std::to_string(z));
            }
        for (int f = 0; f < 8; ++f) m->fld[f][z] = tok[4 + f];
        const double g_det = tok[33];
        bn += d_v * g_det * std::pow(m->fld[1][z] / m->fld[0][z] * u.theta_e_unit, 2.);
        vol += d_v * g_det;
    }
    m->bias_norm = bn / vol;
    m->rh = 1.0 + std::sqrt(1.0 - h.a * h.a);
    m->x1_min = std::log(m->rh);
    *out = m;
    return 0;
}

void grm_model_free(grm_model *m) { delete m; }

/* init(): harm_model.cpp:234-240 */
/* library-internal device builders (csrc/grm_tables.hip) */
int grm_tables_hot_k2_device(int device, const double c[13], const double *grid, double *hot, double *k2, float *ms,
                             std::string &err);
int grm_tables_nint_device(int device, const double c[13], const double *ftab, const double *weight, double *nint,
                           double *dndlnu_max, float *ms, std::string &err);

namespace {
int model_init(grm_model *m, int n_threads, int device);
}

int grm_model_init(grm_model *m, int n_threads) { return model_init(m, n_threads, -1); }

int grm_model_init_device(grm_model *m, int n_threads, int device) {
    if (device < 0) return set_err("grm_model_init_device: device < 0");
    return model_init(m, n_threads, device);
}

namespace {
int model_init(grm_model *m, int n_threads, int device) {
    if (!m) return set_err("null model");
    if (n_threads < 1) n_threads = default_threads();
    const int n1 = m->n1(), n2 = m->n2();
    const size_t nz = (size_t)n1 * n2;
    /* geometry (:242-266) */
    m->gcov.assign(nz * 16, 0.0);
    m->gcon0.assign(nz * 4, 0.0);
    m->det.assign(nz, 0.0);
    parallel_for(n1, n_threads, [&](int i) {
        for (int j = 0; j < n2; ++j) {
            double x[4];
            zone_coord(m, i, j, x);
            const size_t z = (size_t)i * n2 + j;
            metric_cov(m, x, &m->gcov[z * 16]);
            metric_con_row0(m, x, &m->gcon0[z * 4]);
            m->det[z] = std::sqrt(std::abs(det4(&m->gcov[z * 16])));
        }
    });
    /* device builders' constants (csrc/grm_tables.hip TableConsts) */
    const grm_header &h = m->hdr;
    const double nfac = h.dx[1] * h.dx[2] * h.dx[3] * m->units.l_unit * m->units.l_unit * m->units.l_unit * kSqrt2 *
                        EE * EE * EE / (27.0 * ME * CL * CL) * (1.0 / HPL);
    const double tc[13] = {K.hc_l_min_w, K.hc_d_l_w, K.hc_l_min_t, K.hc_d_l_t, K.jnu_l_min_t, K.jnu_d_l_t,
                           K.jnu_l_min_k, K.jnu_d_l_k, K.l_nu_min, K.d_l_nu, K.l_b_min, K.d_l_b, nfac};
    m->table_ms = 0.0;
    /* hotcross table (hotcross.cpp:60-79): one quadrature column per temperature */
    m->hot.assign((size_t)(HC_N_W + 1) * (HC_N_T + 1), 0.0);
    m->ftab.assign(NSAMP + 1, 0.0);
    m->k2.assign(NSAMP + 1, 0.0);
    if (device >= 0) { /* hotcross and K2 on the GPU */
        std::string err;
        float ms = 0.f;
        std::vector<double> grid(HC_N_W + 1 + HC_N_T + 1);
        for (int ii = 0; ii <= HC_N_W; ++ii) grid[ii] = std::pow(10.0, K.hc_l_min_w + ii * K.hc_d_l_w);
        for (int jj = 0; jj <= HC_N_T; ++jj) grid[HC_N_W + 1 + jj] = std::pow(10.0, K.hc_l_min_t + jj * K.hc_d_l_t);
        if (grm_tables_hot_k2_device(device, tc, grid.data(), m->hot.data(), m->k2.data(), &ms, err)) return set_err(err);
        m->table_ms += ms;
    } else
    parallel_for(HC_N_T + 1, n_threads, [&](int jj) {
        const double l_t = K.hc_l_min_t + jj * K.hc_d_l_t;
        const double th = std::pow(10.0, l_t);
        const HotColumn col = hot_column(th);
        for (int ii = 0; ii <= HC_N_W; ++ii) {
            const double l_w = K.hc_l_min_w + ii * K.hc_d_l_w;
            m->hot[(size_t)ii * (HC_N_T + 1) + jj] = std::log10(hot_sigma(std::pow(10.0, l_w), th, col));
        }
    });
    /* emission tables (jnu_mixed.cpp:57-73) */
    try {
        parallel_for(NSAMP + 1, n_threads, [&](int q) {
            const double k = std::exp(q * K.jnu_d_l_k + K.jnu_l_min_k);
            auto integrand = [k](double th) {
                const double s = std::sin(th), x = k / s;
                if (s < 1.0e-150 || x > 2.0e8) return 0.0;
                return s * s * std::pow(std::sqrt(x) + JNU_CST * std::pow(x, 1.0 / 6.0), 2.0) *
                       std::exp(-std::pow(x, 1.0 / 3.0));
            };
            m->ftab[q] = std::log(4 * kPi * adaptive_gk61(integrand, 0, kPi / 2.0, 0.0, 1.0e-6, 1000));
            if (device < 0) {
                const double tq = std::exp(q * K.jnu_d_l_t + K.jnu_l_min_t);
                m->k2[q] = std::log(std::cyl_bessel_k(2, 1.0 / tq));
            }
        });
    } catch (const std::exception &ex) {
        return set_err(ex.what());
    }
    /* weight table (:268-306): each frequency bin sums zones in reference order */
    std::vector<double> nu(NSAMP + 1);
    for (int q = 0; q <= NSAMP; ++q) nu[q] = std::exp(q * K.d_l_nu + K.l_nu_min);
    const double s_fac = h.dx[1] * h.dx[2] * h.dx[3] * m->units.l_unit * m->units.l_unit * m->units.l_unit;
    std::vector<Fluid> zf(nz);
    std::vector<double> zfac(nz, 0.0);
    std::vector<char> zok(nz, 0);
    parallel_for(n1, n_threads, [&](int i) {
        for (int j = 0; j < n2; ++j) {
            const size_t z = (size_t)i * n2 + j;
            zf[z] = zone_fluid(m, i, j);
            if (zf[z].n_e == 0.0 || zf[z].theta_e < THETA_E_MIN) continue;
            const double k2 = k2_eval(m, zf[z].theta_e);
            zfac[z] = (JCST * zf[z].n_e * zf[z].b * zf[z].theta_e * zf[z].theta_e / k2) * s_fac * m->det[z];
            zok[z] = 1;
        }
    });
    m->weight.assign(NSAMP + 1, 0.0);
    parallel_for(NSAMP + 1, n_threads, [&](int q) {
        double sum = 0.0;
        for (size_t z = 0; z < nz; ++z)
            if (zok[z]) sum += zfac[z] * f_eval(m, zf[z].theta_e, zf[z].b, nu[q]);
        m->weight[q] = std::log(sum / (HPL * m->photon_n));
    });
    /* nint table (:308-338) */
    m->nint.assign(NINT + 1, 0.0);
    m->dndlnu_max.assign(NINT + 1, 0.0);
    if (device >= 0) {
        std::string err;
        float ms = 0.f;
        if (grm_tables_nint_device(device, tc, m->ftab.data(), m->weight.data(), m->nint.data(), m->dndlnu_max.data(),
                                   &ms, err))
            return set_err(err);
        m->table_ms += ms;
        m->inited = true;
        return 0;
    }
    parallel_for((NINT + 1 + 255) / 256, n_threads, [&](int blk) {
        for (int i = blk * 256; i < std::min(NINT + 1, (blk + 1) * 256); ++i) {
            double s = 0.0, dmax = 0.0;
            const double b_mag = std::exp(i * K.d_l_b + K.l_b_min);
            for (int q = 0; q < NSAMP; ++q) {
                const double dn = f_eval(m, 1.0, b_mag, std::exp(q * K.d_l_nu + K.l_nu_min)) /
                                  (std::exp(m->weight[q]) + 1.0e-100);
                if (dn > dmax) dmax = dn;
                s += K.d_l_nu * dn;
            }
            s *= nfac;
            m->nint[i] = std::log(s);
            m->dndlnu_max[i] = std::log(dmax);
        }
    });
    m->inited = true;
    return 0;
}
} /* namespace */

double grm_model_table_ms(const grm_model *m) { return m ? m->table_ms : 0.0; }

void grm_model_header(const grm_model *m, grm_header *h) { *h = m->hdr; }
void grm_model_units(const grm_model *m, grm_units *u) { *u = m->units; }
void grm_model_scalars(const grm_model *m, double out[5]) {
    out[0] = m->bias_norm;
    out[1] = m->x1_min;
    out[2] = m->max_tau_scatt;
    out[3] = m->d_tau_k;
    out[4] = m->rh;
}
const double *grm_model_field(const grm_model *m, int which) {
    return (which >= 0 && which < 8) ? m->fld[which].data() : nullptr;
}
const double *grm_model_table(const grm_model *m, int which) {
    switch (which) {
    case 0: return m->hot.data();
    case 1: return m->k2.data();
    case 2: return m->ftab.data();
    case 3: return m->weight.data();
    case 4: return m->nint.data();
    case 5: return m->dndlnu_max.data();
    case 6: return m->det.data();
    default: return nullptr;
    }
}

int grm_model_zone_weights(const grm_model *m, double *out) {
    if (!m || !m->inited || !out) return set_err("model not initialised");
    const int n2 = m->n2();
    parallel_for(m->n1(), default_threads(), [&](int i) {
        for (int j = 0; j < n2; ++j) {
            double nz, dm;
            zone_budget(m, i, j, nz, dm);
            out[(size_t)i * n2 + j] = nz;
        }
    });
    return 0;
}

int64_t grm_model_emit(grm_model *m, uint64_t seed, int64_t z0, int64_t z1, grm_init_photon *out, size_t cap,
                       int n_threads) {
    return grm_model_emit_strided(m, seed, z0, z1, 1, out, cap, n_threads);
}

int64_t grm_model_emit_strided(grm_model *m, uint64_t seed, int64_t z0, int64_t z1, int64_t stride, grm_init_photon *out,
                               size_t cap, int n_threads) {
    if (!m || !m->inited) {
        set_err("model not initialised");
        return -1;
    }
    const int64_t nz = (int64_t)m->n1() * m->n2();
    if (z1 < 0 || z1 > nz) z1 = nz;
    if (z0 < 0) z0 = 0;
    if (z0 >= z1) return 0;
    if (stride < 1) {
        set_err("emit: stride < 1");
        return -1;
    }
    if (n_threads < 1) n_threads = default_threads();
    const int64_t n = (z1 - z0 + stride - 1) / stride; /* zones z0 + q * stride */
    std::vector<int> cnt((size_t)n);
    const int CH = 256;
    parallel_for((int)((n + CH - 1) / CH), n_threads, [&](int c) {
        for (int64_t q = (int64_t)c * CH; q < std::min<int64_t>(n, (int64_t)(c + 1) * CH); ++q) {
            const int64_t z = z0 + q * stride;
            cnt[(size_t)q] = zone_count(m, seed, (int)(z / m->n2()), (int)(z % m->n2()));
        }
    });
    std::vector<int64_t> off((size_t)n + 1, 0);
    for (int64_t q = 0; q < n; ++q) off[(size_t)q + 1] = off[(size_t)q] + cnt[(size_t)q];
    const int64_t total = off[(size_t)n];
    if (!out) return total;
    if ((size_t)total > cap) {
        set_err("emit: output capacity " + std::to_string(cap) + " < " + std::to_string(total));
        return -1;
    }
    parallel_for((int)((n + CH - 1) / CH), n_threads, [&](int c) {
        for (int64_t q = (int64_t)c * CH; q < std::min<int64_t>(n, (int64_t)(c + 1) * CH); ++q) {
            if (cnt[(size_t)q] == 0) continue;
            const int64_t z = z0 + q * stride;
            grm_emit_zone r;
            zone_record(m, (int)(z / m->n2()), (int)(z % m->n2()), r);
            emit_zone(m, r, seed, (uint64_t)z, cnt[(size_t)q], out + off[(size_t)q]);
        }
    });
    return total;
}

int grm_model_zone_table(const grm_model *m, int64_t z0, int64_t z1, grm_emit_zone *out, int n_threads) {
    if (!m || !m->inited || !out) return set_err("zone table: model not initialised");
    const int64_t nz = (int64_t)m->n1() * m->n2();
    if (z1 < 0 || z1 > nz) z1 = nz;
    if (z0 < 0) z0 = 0;
    const int64_t n = z1 - z0;
    if (n <= 0) return 0;
    const int CH = 256;
    parallel_for((int)((n + CH - 1) / CH), n_threads, [&](int c) {
        for (int64_t q = (int64_t)c * CH; q < std::min<int64_t>(n, (int64_t)(c + 1) * CH); ++q) {
            const int64_t z = z0 + q;
            zone_record(m, (int)(z / m->n2()), (int)(z % m->n2()), out[q]);
        }
    });
    return 0;
}

int grm_engine_emit_setup_from_model(grm_engine *e, const grm_model *m) {
    if (!e) return -1;
    if (!m || !m->inited) return set_err("emit setup: model not initialised");
    const int64_t nz = (int64_t)m->n1() * m->n2();
    std::vector<grm_emit_zone> zt((size_t)nz);
    if (grm_model_zone_table(m, 0, nz, zt.data(), 0)) return -1;
    return grm_engine_emit_setup(e, zt.data(), nz, m->weight.data(), m->ftab.data());
}

/* report_spectrum (harm_model.cpp:416-471, d_omega_func :532-536) */
int grm_write_spectrum(const grm_model *m, const grm_spectrum_cell *spec, const char *path, double out2[2]) {
    if (!m || !spec) return set_err("null argument");
    const grm_header &h = m->hdr;
    const double dx2 = (h.x_stop[2] - h.x_start[2]) / (2 * GRM_N_TH_BINS);
    auto d_omega = [&](double a, double b) {
        return 2.0 * kPi *
               (-std::cos(kPi * b + 0.5 * (1.0 - h.h_slope) * std::sin(2 * kPi * b)) +
                std::cos(kPi * a + 0.5 * (1.0 - h.h_slope) * std::sin(2 * kPi * a)));
    };
    FILE *fp = path ? std::fopen(path, "w") : nullptr;
    if (path && !fp) return set_err(std::string("Cannot open file ") + path);
    double lum = 0.0, maxt = 0.0;
    for (int i = 0; i < GRM_N_E_BINS; ++i) {
        if (fp) std::fprintf(fp, "%10.5g ", (i * SPEC_D_L_E + K.spec_l_e_0) / kLn10);
        for (int j = 0; j < GRM_N_TH_BINS; ++j) {
            const grm_spectrum_cell &s = spec[j * GRM_N_E_BINS + i];
            const double dom = 2.0 * d_omega(j * dx2, (j + 1) * dx2);
            double nu_lnu = (ME * CL * CL) * (4.0 * kPi / dom) * (1.0 / SPEC_D_L_E);
            nu_lnu *= s.de_dle;
            nu_lnu /= L_SUN;
            const double ts = s.tau_scatt / (s.dn_dle + EPS);
            if (fp)
                std::fprintf(fp, "%10.5g %10.5g %10.5g %10.5g %10.5g %10.5g ", nu_lnu, s.tau_abs / (s.dn_dle + EPS), ts,
                             s.x1i_av / (s.dn_dle + EPS), std::sqrt(std::abs(s.x2i_sq / (s.dn_dle + EPS))),
                             std::sqrt(std::abs(s.x3f_sq / (s.dn_dle + EPS))));
            if (ts > maxt) maxt = ts;
            lum += nu_lnu * dom * SPEC_D_L_E;
        }
        if (fp) std::fprintf(fp, "\n");
    }
    if (fp) std::fclose(fp);
    if (out2) {
        out2[0] = lum;
        out2[1] = maxt;
    }
    return 0;
}

int grm_write_spectrum_stats(const grm_model *m, const grm_spectrum_cell *spec, const char *path) {
    if (!m || !spec || !path) return set_err("null argument");
    FILE *fp = std::fopen(path, "w");
    if (!fp) return set_err(std::string("Cannot open file ") + path);
    std::fprintf(fp, "# log10(E/me c^2); per theta bin 0..%d: nph dn_dle de_dle\n", GRM_N_TH_BINS - 1);
    for (int i = 0; i < GRM_N_E_BINS; ++i) {
        std::fprintf(fp, "%.17g", (i * SPEC_D_L_E + K.spec_l_e_0) / kLn10);
        for (int j = 0; j < GRM_N_TH_BINS; ++j) {
            const grm_spectrum_cell &s = spec[j * GRM_N_E_BINS + i];
            std::fprintf(fp, " %.17g %.17g %.17g", s.nph, s.dn_dle, s.de_dle);
        }
        std::fprintf(fp, "\n");
    }
    const bool ok = std::fclose(fp) == 0;
    return ok ? 0 : set_err(std::string("write failed: ") + path);
}

int grm_engine_create_from_model(const grm_model *m, int device, grm_engine **out) {
    if (!m || !m->inited) return set_err("model not initialised");
    const double *f[8];
    for (int q = 0; q < 8; ++q) f[q] = m->fld[q].data();
    const double sc[4] = {m->bias_norm, m->x1_min, m->max_tau_scatt, m->d_tau_k};
    return grm_engine_create(&m->hdr, f, &m->units, m->hot.data(), m->k2.data(), sc, device, out);
}

} /* extern "C" */
