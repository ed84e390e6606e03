/*
 * ref_harness.cpp -- thin C wrappers around the REFERENCE's own compiled
 * sources (cuda_grmonty/{tetrads,proba,monty_rand,integration}.cpp, compiled
 * in place from /root/reference by oracle/Makefile into oracle/_ref/).  No
 * reference source is copied: this file only calls the reference API so the
 * oracle restatement can be checked bit-for-bit against it.
 *
 * Only these four translation units are buildable here: the rest of the
 * reference (harm_model/radiation/hotcross/jnu_mixed/main) includes spdlog and
 * std::format, which this image lacks, and is therefore unbuildable.
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <numbers>

#include "cuda_grmonty/integration.hpp"
#include "cuda_grmonty/monty_rand.hpp"
#include "cuda_grmonty/ndarray.hpp"
#include "cuda_grmonty/proba.hpp"
#include "cuda_grmonty/tetrads.hpp"

extern "C" {

void ref_rng_init(int seed) { monty_rand::init(seed); }
double ref_uniform(void) { return monty_rand::uniform(); }
double ref_chi_sq(int dof) { return monty_rand::chi_sq(dof); }

void ref_sample_electron(const double k_in[4], double p_out[4], double theta_e) {
    double k[4] = {k_in[0], k_in[1], k_in[2], k_in[3]};
    double p[4];
    proba::sample_electron_distr_p(k, p, theta_e);
    std::memcpy(p_out, p, sizeof(p));
}
double ref_sample_klein_nishina(double k0) { return proba::sample_klein_nishina(k0); }
double ref_sample_thomson(void) { return proba::sample_thomson(); }
void ref_sample_rand_dir(double out[3]) {
    auto [x, y, z] = proba::sample_rand_dir();
    out[0] = x;
    out[1] = y;
    out[2] = z;
}
double ref_sample_y(double theta_e) { return proba::sample_y_distr(theta_e); }
double ref_sample_mu(double beta_e) { return proba::sample_mu_distr(beta_e); }

void ref_make_tetrad(const double u_con_in[4], const double trial_in[4], const double g_cov_in[16], double e_con_out[16],
                     double e_cov_out[16]) {
    double u_con[4], trial[4], e_con[4][4], e_cov[4][4];
    std::memcpy(u_con, u_con_in, sizeof(u_con));
    std::memcpy(trial, trial_in, sizeof(trial));
    ndarray::NDArray<double, 2> g({4, 4});
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) g(i, j) = g_cov_in[i * 4 + j];
    tetrads::make_tetrad(u_con, trial, g, e_con, e_cov);
    std::memcpy(e_con_out, e_con, sizeof(e_con));
    std::memcpy(e_cov_out, e_cov, sizeof(e_cov));
}

void ref_coordinate_to_tetrad(const double e_cov_in[16], const double k_in[4], double out[4]) {
    double e_cov[4][4], k[4], kt[4];
    std::memcpy(e_cov, e_cov_in, sizeof(e_cov));
    std::memcpy(k, k_in, sizeof(k));
    tetrads::coordinate_to_tetrad(e_cov, k, kt);
    std::memcpy(out, kt, sizeof(kt));
}

void ref_tetrad_to_coordinate(const double e_con_in[16], const double kt_in[4], double out[4]) {
    double e_con[4][4], kt[4], k[4];
    std::memcpy(e_con, e_con_in, sizeof(e_con));
    std::memcpy(kt, kt_in, sizeof(kt));
    tetrads::tetrad_to_coordinate(e_con, kt, k);
    std::memcpy(out, k, sizeof(k));
}

/* same integrand codes as grmo_gk61 (0..9) */
double ref_gk61(int which, double a, double b, double eps_abs, double eps_rel, int max_iv) {
    std::function<double(double)> f;
    switch (which) {
    case 0: f = [](double) { return 1.0; }; break;
    case 1: f = [](double x) { return 2.0 * x + 1.0; }; break;
    case 2: f = [](double x) { return -x * x + 1.0; }; break;
    case 3: f = [](double x) { return std::sin(x); }; break;
    case 4: f = [](double x) { return std::abs(x - 0.3); }; break;
    case 5: f = [](double x) { return std::sqrt(x); }; break;
    case 6: f = [](double x) { return std::log(x); }; break;
    case 7: f = [](double x) { return std::sin(20 * x); }; break;
    case 8: f = [](double x) { return 1.0 / (1.0 + 1000.0 * (x - 0.5) * (x - 0.5)); }; break;
    case 9: f = [](double x) { return (x < 0.5) ? 0.0 : 1.0; }; break;
    default: f = [](double x) { return x; }; break;
    }
    try {
        return integration::gauss_kronrod_61(f, a, b, eps_abs, eps_rel, max_iv);
    } catch (...) {
        return std::nan("");
    }
}

} /* extern "C" */
