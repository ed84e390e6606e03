// Host check of cuda-grmonty_amd/csrc/grm_crlog.h (the device table builders' log / log10): compiled
// with g++, the header's correction starts from glibc's log itself, and the results are compared
// with glibc's log and log10 on random arguments and on the Klein-Nishina arguments 1 + 2w of the
// hotcross w range.  Prints: n, cr_log != log, grm_log10 != log10, cr_log's mismatches that glibc
// misrounds (checked by the caller against a high-precision log).
#include <cmath>
#include <cstdio>
#include <random>

#define GRM_CR_FN inline
#define GRM_CR_LOG(x) std::log(x)
using std::fma;
using std::ldexp;
using std::rint;
#include "grm_crlog.h"

int main() {
    std::mt19937_64 g(7);
    long n = 0, bad_log = 0, bad_l10 = 0;
    for (int t = 0; t < 400000; ++t) {
        double x;
        if (t % 2)
            x = std::exp(std::uniform_real_distribution<double>(-700.0, 700.0)(g));
        else
            x = 1.0 + 2.0 * std::pow(10.0, std::uniform_real_distribution<double>(-3.0, 6.0)(g));
        ++n;
        const double a = grm_cr::cr_log(x), b = grm_cr::grm_log10(x);
        if (a != std::log(x)) {
            ++bad_log;
            std::printf("log %a %a %a\n", x, a, std::log(x));
        }
        if (b != std::log10(x)) ++bad_l10;
    }
    /* special arguments: zero, subnormal, negative, infinities, NaN -- grm_log10 as glibc's log10 */
    long bad_special = 0;
    const double sp[] = {0.0, -0.0, 4.9e-324, 1.0e-310, -1.0, -INFINITY, INFINITY, NAN};
    for (double x : sp) {
        const double a = grm_cr::grm_log10(x), b = std::log10(x);
        if (!(a == b || (std::isnan(a) && std::isnan(b)))) {
            ++bad_special;
            std::printf("special %a %a %a\n", x, a, b);
        }
    }
    std::printf("n %ld log_diff %ld log10_diff %ld special_bad %ld\n", n, bad_log, bad_l10, bad_special);
    return 0;
}
