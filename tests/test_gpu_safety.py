"""Robustness of the transport launch (grm_engine.hip):

1. A photon whose position turns NaN ends at once and leaves the results of every other photon unchanged --
   in the reference it loops to max_n_step (harm_model.cpp:1058-1063) and is never recorded
   (:1066, record_super_photon :1291-1295), so ending it early is output-equivalent.
2. The per-launch watchdog (GRM_OPT_WATCHDOG_MS) abandons a launch that runs too long, reports it as
   an error with the abandoned photons' state, and the engine stays usable afterwards.
3. The kernel-argument guard of track_kernel (kargs_check, grm_engine.hip): the launch's arguments
   are read in the loop through the kernarg segment laid out as struct KArgs; every wave compares
   that view with the by-value parameters at entry.  A normal call reports it clean; with the
   failure injected (GRM_OPT_KARG_TEST) the call fails with the reason, tracks nothing, and the
   engine is usable afterwards.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frozen(G, eng):
    eng.reset()
    eng.set_option(G.OPT_SEED, 123)
    eng.set_option(G.OPT_ID_BASE, 0)
    eng.set_option(G.OPT_BIAS_MODE, 1)  # bias frozen at the counters of the call start (just reset)


def test_nan_photon_is_inert(model64):
    import grmonty_amd as G
    full = model64.emit(seed=123)
    ph = full[:4000].copy()
    eng = G.Engine(model64, device=0)
    _frozen(G, eng)
    eng.track(ph)
    spec_a, nr_a, ns_a, _ = eng.finish()
    nan_a = eng.stats()["n_nan_photons"]
    # the same batch plus one photon on the polar axis at the end (ids of the others unchanged): the
    # connection divides by sin(theta) = 0 there (harm_model.cpp:1436-1569), so its k and then its x
    # turn NaN on the first steps (NaN inputs themselves are rejected at set-up, :895-903)
    bad = full[np.flatnonzero((full["x"][:, 1] > 1.0) & (full["x"][:, 1] < 2.5))[:1]].copy()  # outside the horizon
    bad["x"][0, 2] = 0.0
    bad["w"] = 1.0e40  # above weight_min: no roulette at the first stop test
    _frozen(G, eng)
    eng.track(np.concatenate([ph, bad]))
    spec_b, nr_b, ns_b, _ = eng.finish()
    st = eng.stats()
    assert st["n_nan_photons"] == nan_a + 1
    assert st["n_abandoned"] == 0
    assert (nr_a, ns_a) == (nr_b, ns_b)
    for f in ("dn_dle", "de_dle", "nph", "nscatt"):
        np.testing.assert_allclose(spec_b[f], spec_a[f], rtol=1e-12, atol=0)


def test_watchdog_abandons_and_recovers(model64):
    import grmonty_amd as G
    ph = model64.emit(seed=123)
    eng = G.Engine(model64, device=0)
    eng.reset()
    eng.set_option(G.OPT_WARMUP, 0)
    eng.set_option(G.OPT_WATCHDOG_MS, 1)
    big = np.concatenate([ph] * max(1, 400_000 // len(ph)))
    with pytest.raises(RuntimeError, match="watchdog"):
        eng.track(big)
    st = eng.stats()
    assert st["n_abandoned"] > 0
    stuck = eng.debug_stuck()
    assert 0 < len(stuck) <= min(256, st["n_abandoned"])
    assert np.all(np.isfinite(stuck[:, 0])) and np.all(stuck[:, 1] >= 0)  # photon id, n_step
    # back to the default limit: a normal call completes
    eng.set_option(G.OPT_WATCHDOG_MS, 60000)
    eng.reset()
    eng.track(ph[np.random.default_rng(1).permutation(len(ph))[:4000]])
    _, nr, _, _ = eng.finish()
    assert eng.stats()["n_abandoned"] == 0 and nr > 0


def test_kernel_argument_guard(model64):
    import grmonty_amd as G
    full = model64.emit(seed=123)
    ph = full[np.random.default_rng(5).permutation(len(full))[:3000]]  # all radii (zone order starts inside)
    eng = G.Engine(model64, device=0)
    _frozen(G, eng)
    eng.track(ph)
    assert eng.debug_counters()["karg_bad"] == 0
    _, nr0, _, _ = eng.finish()
    assert nr0 > 0
    _frozen(G, eng)
    eng.set_option(G.OPT_KARG_TEST, 1)
    with pytest.raises(RuntimeError, match="kernel-argument"):
        eng.track(ph)
    c = eng.debug_counters()
    assert c["karg_bad"] > 0 and c["n_steps"] == 0 and c["n_tracked"] == 0
    eng.set_option(G.OPT_KARG_TEST, 0)
    _frozen(G, eng)
    eng.track(ph)
    _, nr1, _, _ = eng.finish()
    assert nr1 == nr0 and eng.debug_counters()["karg_bad"] == 0
    eng.close()
