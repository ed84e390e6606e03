"""BASELINE.json's other configs as GPU parity cases (the headline, configs[1], is bench.py's):

- configs[4], a 512 x 512 HARM grid (the HBM-interpolation stress): photon-by-photon against the
  oracle with the bias frozen, as tests/test_gpu_transport.py does on 64 x 64;
- configs[2], photon_n = 1e7 on the 192 x 192 dump019-class grid (145 M superphotons, the
  scattered-child spawn / compaction stress): size-independent properties -- no child lost, counters
  consistent, and the luminosity estimate equal to the photon_n = 1e6 one within its Monte Carlo
  spread (superphoton weights scale as 1 / photon_n, harm_model.cpp:1337-1389).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dump512(dump_dir):
    from grmonty_amd.synth_dump import write_dump
    return write_dump(os.path.join(dump_dir, "synth512.dump"), 512, 512)


@pytest.fixture(scope="module")
def dump192(dump_dir):
    from grmonty_amd.synth_dump import write_dump
    return write_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)


def test_grid512_photon_by_photon(dump512):
    import grmonty_amd as G
    import oracle_py as O
    model = G.Model.load(dump512, photon_n=20000).init(8)
    oracle = O.OracleModel(dump512, photon_n=20000)
    oracle.init(8)
    ph = model.emit(seed=123)
    rng = np.random.default_rng(7)
    sel = ph[rng.permutation(len(ph))[:600]]
    oracle.reset()
    tr_o = oracle.track(sel, rng_mode=1, seed=123, id_base=0, frozen=True, scatt0=1000, rec0=2000,
                        max_tau0=model.scalars()["max_tau_scatt"], trace_cap=2_000_000)
    spec_o = oracle.spectrum()
    eng = G.Engine(model, device=0)
    eng.reset()
    eng.set_option(G.OPT_SEED, 123)
    eng.set_option(G.OPT_ID_BASE, 0)
    eng.set_option(G.OPT_BIAS_MODE, 1)
    eng.set_option(G.OPT_FROZEN_SCATT, 1000)
    eng.set_option(G.OPT_FROZEN_REC, 2000)
    eng.set_option(G.OPT_FROZEN_MAXTAU, int(np.float64(model.scalars()["max_tau_scatt"]).view(np.int64)))
    eng.set_option(G.OPT_TRACE_CAP, 2_000_000)
    eng.track(sel)
    tr_g = eng.trace(2_000_000)
    spec_g = eng.finish()[0]
    st = eng.stats()
    assert st["n_dropped"] == 0 and st["n_primaries"] == len(sel)
    from parity_util import MIN_MATCH, check_spectrum_cells, trace_match
    n_o, n_g, match, bad = trace_match(tr_o, tr_g)
    n_cmp, n_excl = check_spectrum_cells(spec_o, spec_g, tr_o, tr_g, bad)
    print(f"512^2: oracle ends {n_o} device ends {n_g} matching {match / n_o:.4f}; spectrum cells compared "
          f"(12 fields) {n_cmp}, excluded {n_excl}")
    assert match / n_o >= MIN_MATCH


def test_photon_n_1e7_consistency(dump192):
    import grmonty_amd as G
    lum = {}
    for pn in (1e6, 1e7):
        model = G.Model.load(dump192, photon_n=pn).init(8)
        eng = G.Engine(model, device=0)
        eng.emit_setup(model)
        eng.reset()
        p, n = eng.emit(seed=123)
        eng.track_device(p, n)
        spec, n_rec, n_scatt, _ = eng.finish()
        st = eng.stats()
        assert st["n_dropped"] == 0 and st["n_abandoned"] == 0
        assert st["n_primaries"] == n
        assert st["n_tracked"] == st["n_primaries"] + st["n_children"]
        assert int(round(spec["nph"].sum())) == n_rec
        lum[pn] = spec["de_dle"].sum()
        print(f"photon_n {pn:.0e}: {n} emitted, {st['n_tracked']} tracked, {n_rec} recorded, "
              f"{n_scatt} scattered, sum w e = {lum[pn]:.6e}, overflow {st['n_overflow']}")
        del eng
    assert n > 1.0e8
    assert abs(lum[1e7] - lum[1e6]) <= 0.05 * lum[1e6]
