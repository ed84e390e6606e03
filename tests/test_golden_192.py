"""Headline-scale statistical fixtures (tests/golden/oracle_synth192_pn1e5.*, tools/make_golden_192.py):
the oracle run_simulation runs (reference CPU semantics: serial, mt19937, live adaptive bias) on
the 192x192 dump019-class synthetic dump at photon_n = 1e5 (BASELINE configs[0]).

These tests calibrate the statistic the GPU parity test (tests/test_gpu_parity_192.py) applies to
the device: independent reference-semantics runs must pass the binned Kish-N KS test on nu L_nu
against each other, per theta bin and summed: the fraction of the (pairs x 7) statistics over the
test's own threshold (alpha = 1e-4) and over alpha = 1e-3 must stay near those rates (the maximum over
thousands of pairs would exceed either by chance)."""
import json
import os

import numpy as np
import pytest

from spectrum_stats import binned_ks, ks_crit

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = [os.path.join(HERE, "golden", f"oracle_synth192_{p}") for p in ("pn1e5", "pn1e6")]


@pytest.mark.parametrize("G", FIXTURES, ids=["pn1e5", "pn1e6"])
def test_oracle_seeds_pass_binned_ks(G):
    g = np.load(G + ".npz")
    cells = g["cells"]
    worst, over, over4, tot = 0.0, 0, 0, 0
    for i in range(len(cells)):
        for j in range(i + 1, len(cells)):
            for th in [None, 0, 1, 2, 3, 4, 5]:
                d, n1, n2 = binned_ks(cells[i], cells[j], th)
                worst = max(worst, d / ks_crit(n1, n2, 1e-4))
                over4 += d >= ks_crit(n1, n2, 1e-4)
                over += d >= ks_crit(n1, n2, 1e-3)
                tot += 1
    print(f"{len(cells)} runs: worst D / crit(alpha=1e-4) over {tot} statistics: {worst:.2f}; over crit(1e-4): "
          f"{over4} of {tot} (nominal {1e-4 * tot:.1f}); over crit(1e-3): {over} of {tot} (nominal {1e-3 * tot:.1f})")
    # the statistic is calibrated when independent reference runs exceed its critical values at about
    # the nominal rates (the maximum over all pairs is not a calibration: 102 runs make 36 k statistics,
    # ~3.6 of which exceed crit(1e-4) by chance)
    assert over4 <= max(2, 5e-4 * tot)
    assert over <= max(2, 0.01 * tot)


@pytest.mark.parametrize("G", FIXTURES, ids=["pn1e5", "pn1e6"])
def test_fixture_consistency(G):
    g = np.load(G + ".npz")
    s = json.load(open(G + ".json"))
    cnt = g["counters"]  # created, scattered, recorded, steps
    for k, run in enumerate(s["runs"]):
        assert run["seed"] == int(g["seeds"][k])
        assert (run["created"], run["scattered"], run["recorded"], run["steps"]) == tuple(int(x) for x in cnt[k])
        # every recorded superphoton lands in exactly one cell (record_super_photon, harm_model.cpp:1306-1333)
        assert int(round(g["cells"][k][:, 0].sum())) == run["recorded"]
    spec = g["spectrum123"]  # [6, 200, 13]: nph field (index 2) of seed 123
    assert int(round(spec[:, :, 2].sum())) == s["runs"][0]["recorded"]
    np.testing.assert_allclose(spec[:, :, 1].reshape(-1), g["cells"][0][:, 3], rtol=1e-9)


def test_lag_emulator_fixture():
    """The concurrency emulator's runs (tests/golden/lag_emulator_synth192_pn1e5.json): the serial
    setting -- the reference scheduled serially, on the device's emission and Philox streams -- and
    the device-like setting both agree with the reference's own mt19937 runs within Z_MAX combined
    standard errors on every counter: the RNG streams and the concurrent scheduling of the live bias
    move the counters by ~1-2 %, well inside the device test's bar (tests/test_gpu_parity_192.py)."""
    from spectrum_stats import welch_z
    emu = json.load(open(os.path.join(HERE, "golden", "lag_emulator_synth192_pn1e5.json")))
    ora = json.load(open(os.path.join(HERE, "golden", "oracle_synth192_pn1e5.json")))["runs"]
    for cfg in ("serial", "device", "device_cap"):
        runs = [r for r in emu["runs"] if r["config"] == cfg]
        assert len(runs) >= 20
        for k in ("recorded", "scattered", "steps", "luminosity"):
            diff, se, z = welch_z([r[k] for r in runs], [r[k] for r in ora])
            assert abs(z) < 4.5, (cfg, k, z)


def test_philox_serial_matches_mt19937_reference():
    """The counter offset settled at the reference level (verdict r05, item 2; CPU only).  The
    emulator's serial configuration is the reference's own scheduling (one photon at a time, children
    depth-first, counters fresh every step) on the device's streams: Philox4x32-10 per photon id,
    53-bit (0, 1] uniforms, chi^2 as -2 ln(prod u) (+ a Box-Muller z^2 for odd dof) -- SURVEY Q4,
    proba.cuh:227-233 -- where the reference uses mt19937 with [0, 1) uniforms and libstdc++'s
    gamma-based chi^2 (monty_rand.cpp:19-31).  If the two constructions differed in law, the serial
    runs would sit off the mt19937 runs; with >= 60 runs on each side every counter and the
    luminosity agree within 3 combined standard errors (measured, 64 vs 102 runs: recorded +0.85 %
    (0.85 SE), scattered +1.14 % (0.83), steps +0.79 % (0.79), L -0.01 % (-0.10); against the first
    60 mt19937 runs +1.00 / +1.30 / +0.92 / -0.05 %).  So the device's
    +1-2 % against the mt19937 fixture is not the streams': it is the concurrency of the live bias
    (the device-scheduled emulator reproduces it, test_lag_emulator_fixture).  Round 5's +2.68 % was
    the first 24 runs' sample."""
    from spectrum_stats import welch_z
    emu = json.load(open(os.path.join(HERE, "golden", "lag_emulator_synth192_pn1e5.json")))
    ora = json.load(open(os.path.join(HERE, "golden", "oracle_synth192_pn1e5.json")))["runs"]
    ser = [r for r in emu["runs"] if r["config"] == "serial"]
    assert len(ser) >= 60 and len(ora) >= 60
    assert len({r["seed"] for r in ser}) == len(ser)
    for k in ("recorded", "scattered", "steps", "luminosity"):
        a, b = [r[k] for r in ser], [r[k] for r in ora]
        diff, se, z = welch_z(a, b)
        print(f"{k:10s} serial Philox {np.mean(a):.6g} ({len(a)} runs)  mt19937 {np.mean(b):.6g} ({len(b)} runs)  "
              f"{diff / np.mean(b):+.2%} = {z:+.2f} SE")
        assert abs(z) < 3.0, (k, z)
