/*
 * grm_main.cpp -- command-line driver with the reference's flags and run sequence
 * (m-torhan/cuda-grmonty main.cpp:20-53, HARMModel::run_simulation harm_model.cpp:340-414):
 *
 *   grmonty_amd --harm_dump_path=DUMP --spectrum_path=OUT [--photon_n=5000000]
 *               [--mass_unit=4e19] [--verbosity=info] [--device=0] [--seed=123]
 *               [--batch=67108864] [--threads=0] [--host_emit] [--stats_path=OUT.stats]
 *
 * read_file -> init -> run_simulation (zone batches emitted and tracked on the GPU; --host_emit:
 * emitted on host threads, batch b+1 overlapping the transport of batch b) -> report_spectrum.
 * "Final rate" = created superphotons / wall time of run_simulation, as in the reference.
 */
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/grmonty_amd.h"

namespace {

int g_verbose = 1; /* 0 warn, 1 info, 2 debug */

void info(const char *msg) {
    if (g_verbose >= 1) std::fprintf(stderr, "[info] %s\n", msg);
}

template <typename... A>
__attribute__((format(printf, 1, 0))) void info(const char *fmt, A... a) {
    if (g_verbose >= 1) {
        std::fprintf(stderr, "[info] ");
        std::fprintf(stderr, fmt, a...);
        std::fprintf(stderr, "\n");
    }
}

bool flag(int argc, char **argv, int &i, const char *name, std::string &val) {
    const size_t n = std::strlen(name);
    const char *a = argv[i];
    if (std::strncmp(a, "--", 2) != 0 || std::strncmp(a + 2, name, n) != 0) return false;
    if (a[2 + n] == '=') {
        val = a + 3 + n;
        return true;
    }
    if (a[2 + n] == 0 && i + 1 < argc) {
        val = argv[++i];
        return true;
    }
    return false;
}

} /* namespace */

int main(int argc, char **argv) {
    long long photon_n = 5000000; /* main.cpp:20 */
    double mass_unit = 4e19;      /* main.cpp:21 */
    std::string dump, spec_path, stats_path, verbosity = "info";
    int device = 0, threads = 0;
    unsigned long long seed = 123; /* consts.hpp:14 */
    long long batch = 1ll << 26; /* photons per zone batch (8.6 GB of emitted photons) */
    bool host_emit = false;
    for (int i = 1; i < argc; ++i) {
        std::string v;
        if (flag(argc, argv, i, "photon_n", v)) photon_n = std::atoll(v.c_str());
        else if (flag(argc, argv, i, "mass_unit", v)) mass_unit = std::atof(v.c_str());
        else if (flag(argc, argv, i, "harm_dump_path", v)) dump = v;
        else if (flag(argc, argv, i, "spectrum_path", v)) spec_path = v;
        else if (flag(argc, argv, i, "verbosity", v)) verbosity = v;
        else if (flag(argc, argv, i, "stats_path", v)) stats_path = v;
        else if (flag(argc, argv, i, "device", v)) device = std::atoi(v.c_str());
        else if (flag(argc, argv, i, "seed", v)) seed = std::strtoull(v.c_str(), nullptr, 10);
        else if (flag(argc, argv, i, "batch", v)) batch = std::atoll(v.c_str());
        else if (flag(argc, argv, i, "threads", v)) threads = std::atoi(v.c_str());
        else if (std::strcmp(argv[i], "--host_emit") == 0) host_emit = true;
        else {
            std::fprintf(stderr, "unknown argument %s\n", argv[i]);
            return 2;
        }
    }
    g_verbose = verbosity == "debug" || verbosity == "trace" ? 2 : (verbosity == "warn" || verbosity == "error" ? 0 : 1);
    info("Parameters:");
    info("\tphoton_n: %lld", photon_n);
    info("\tmass_unit: %g", mass_unit);
    info("\tharm_dump_path: %s", dump.c_str());
    info("\tspectrum_path: %s", spec_path.c_str());

    grm_model *m = nullptr;
    info("Reading file %s", dump.c_str());
    if (grm_model_load(dump.c_str(), (int)photon_n, mass_unit, &m)) {
        std::fprintf(stderr, "[error] %s\n", grm_model_last_error());
        return 1;
    }
    info("Initializing HARM model (tables)");
    if (grm_model_init(m, threads)) {
        std::fprintf(stderr, "[error] %s\n", grm_model_last_error());
        return 1;
    }
    grm_engine *e = nullptr;
    if (grm_engine_create_from_model(m, device, &e)) {
        std::fprintf(stderr, "[error] engine: %s\n", e ? grm_engine_last_error(e) : grm_model_last_error());
        grm_engine_destroy(e);
        return 1;
    }
    grm_engine_set_option(e, GRM_OPT_SEED, (int64_t)seed);

    /* run_simulation: zone-range batches (bounded HBM for the emitted photons), each emitted on the
     * GPU from the zone table and tracked there; --host_emit keeps the host emitter (batch b+1
     * emitted on host threads while batch b is tracked) */
    if (!host_emit && grm_engine_emit_setup_from_model(e, m)) {
        std::fprintf(stderr, "[error] emission setup: %s %s\n", grm_engine_last_error(e), grm_model_last_error());
        return 1;
    }
    info("Starting main loop");
    const auto t0 = std::chrono::steady_clock::now();
    grm_header h;
    grm_model_header(m, &h);
    const long long nzones = (long long)h.n[0] * h.n[1];
    std::vector<double> zw((size_t)nzones);
    grm_model_zone_weights(m, zw.data());
    /* cut the zone walk into ranges of ~batch expected photons */
    std::vector<long long> cuts{0};
    double acc = 0.0;
    for (long long z = 0; z < nzones; ++z) {
        acc += zw[(size_t)z];
        if (acc >= (double)batch) {
            cuts.push_back(z + 1);
            acc = 0.0;
        }
    }
    if (cuts.back() != nzones) cuts.push_back(nzones);
    unsigned long long created = 0;
    std::vector<grm_init_photon> cur, nxt;
    auto emit = [&](size_t b, std::vector<grm_init_photon> &buf) {
        const int64_t n = grm_model_emit(m, seed, cuts[b], cuts[b + 1], nullptr, 0, threads);
        buf.resize((size_t)std::max<int64_t>(n, 0));
        if (n > 0) grm_model_emit(m, seed, cuts[b], cuts[b + 1], buf.data(), buf.size(), threads);
    };
    if (host_emit) emit(0, cur);
    for (size_t b = 0; b + 1 < cuts.size(); ++b) {
        if (host_emit) {
            std::thread prod;
            if (b + 2 < cuts.size()) prod = std::thread(emit, b + 1, std::ref(nxt));
            if (!cur.empty() && grm_engine_track(e, cur.data(), cur.size())) {
                std::fprintf(stderr, "[error] transport: %s\n", grm_engine_last_error(e));
                if (prod.joinable()) prod.join();
                return 1;
            }
            created += cur.size();
            if (prod.joinable()) prod.join();
            std::swap(cur, nxt);
            nxt.clear();
        } else {
            grm_init_photon *d_ph = nullptr;
            uint64_t n = 0;
            if (grm_engine_emit(e, seed, cuts[b], cuts[b + 1], &d_ph, &n) ||
                (n && grm_engine_track_device(e, d_ph, n))) {
                std::fprintf(stderr, "[error] emission/transport: %s\n", grm_engine_last_error(e));
                return 1;
            }
            created += n;
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        info("Rate %.2f ph/s, zone batch %zu/%zu", created / el, b + 1, cuts.size() - 1);
    }
    std::vector<grm_spectrum_cell> spec(GRM_N_TH_BINS * GRM_N_E_BINS);
    uint64_t n_rec = 0, n_scatt = 0;
    double max_tau = 0.0;
    if (grm_engine_finish(e, spec.data(), &n_rec, &n_scatt, &max_tau)) {
        std::fprintf(stderr, "[error] spectrum readback: %s\n", grm_engine_last_error(e));
        return 1;
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    info("Final rate %.2f ph/s", created / el);
    info("Super photons:");
    info("\tcreated: %llu", created);
    info("\tscattered: %llu", (unsigned long long)n_scatt);
    info("\trecorded: %llu", (unsigned long long)n_rec);
    grm_stats st;
    if (grm_engine_stats(e, &st)) {
        std::fprintf(stderr, "[error] engine stats: %s\n", grm_engine_last_error(e));
        return 1;
    }
    info("\ttransport steps: %llu (%.3g steps/s in kernel)", (unsigned long long)st.n_steps,
         st.n_steps / (st.kernel_ms * 1e-3 + 1e-30));
    if (!spec_path.empty()) {
        info("Writing spectrum to file %s", spec_path.c_str());
        double lm[2];
        if (grm_write_spectrum(m, spec.data(), spec_path.c_str(), lm)) {
            std::fprintf(stderr, "[error] %s\n", grm_model_last_error());
            return 1;
        }
        info("\tlumosity: %g", lm[0]);
        info("\tmax_tau_scatt: %g", lm[1]);
    }
    if (!stats_path.empty() && grm_write_spectrum_stats(m, spec.data(), stats_path.c_str())) {
        std::fprintf(stderr, "[error] %s\n", grm_model_last_error());
        return 1;
    }
    grm_engine_destroy(e);
    grm_model_free(m);
    return 0;
}
