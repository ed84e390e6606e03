"""Edge cases of the transport boundary (grm_engine_track / grm_engine_track_device, the reference's
track_super_photons, super_photon.cuh:55-61): empty batches, a single photon, batches that are not a
multiple of a wavefront (64) or a workgroup (512 lanes), and one pass fed as several ragged calls --
photon by photon against the oracle, which tracks the same photons in one call (bias frozen at one
snapshot, the same Philox streams: photon ids run on across the device's calls)."""
import struct

import numpy as np
import pytest

from parity_util import MIN_MATCH, trace_match

pytestmark = pytest.mark.gpu

SNAP = dict(scatt=200, rec=100, maxtau=2e-3)


def _frozen(G, e):
    e.set_option(G.OPT_BIAS_MODE, 1)
    e.set_option(G.OPT_FROZEN_SCATT, SNAP["scatt"])
    e.set_option(G.OPT_FROZEN_REC, SNAP["rec"])
    e.set_option(G.OPT_FROZEN_MAXTAU, struct.unpack("<q", struct.pack("<d", SNAP["maxtau"]))[0])


def test_empty_batches(model64):
    import grmonty_amd as G
    e = G.Engine(model64, device=0)
    e.reset()
    e.track(np.zeros(0, dtype=G.INIT_PHOTON))
    e.track_device(0, 0)
    spec, n_rec, n_scatt, _ = e.finish()
    st = e.stats()
    assert n_rec == 0 and n_scatt == 0 and st["n_tracked"] == 0 and st["n_steps"] == 0
    assert not np.any(spec["nph"]) and not np.any(spec["dn_dle"])
    # the engine tracks normally afterwards
    ph = model64.emit(seed=3)[:100]
    e.track(ph)
    e.finish()
    assert e.stats()["n_primaries"] == 100


@pytest.mark.parametrize("sizes", [(1,), (63,), (65, 1, 447), (513,), (511, 2, 700)],
                         ids=["one", "sub-wave", "ragged-calls", "workgroup+1", "three-calls"])
def test_ragged_batches_photon_by_photon(model64, oracle64, sizes):
    import grmonty_amd as G
    ph = model64.emit(seed=11)
    rng = np.random.default_rng(sum(sizes))
    sel = ph[rng.permutation(len(ph))[:sum(sizes)]]
    oracle64.reset()
    tr_o = oracle64.track(sel, rng_mode=1, seed=123, id_base=0, frozen=True, scatt0=SNAP["scatt"],
                          rec0=SNAP["rec"], max_tau0=SNAP["maxtau"], trace_cap=1_000_000)
    e = G.Engine(model64, device=0)
    e.reset()
    e.set_option(G.OPT_SEED, 123)
    e.set_option(G.OPT_ID_BASE, 0)
    _frozen(G, e)
    e.set_option(G.OPT_TRACE_CAP, 1_000_000)
    a = 0
    for n in sizes:
        e.track(sel[a:a + n])
        a += n
    tr_g = e.trace(1_000_000)
    e.finish()
    st = e.stats()
    n_o, n_g, match, bad = trace_match(tr_o, tr_g)
    print(f"{sizes}: oracle ends {n_o} device ends {n_g} matching {match}; primaries {st['n_primaries']}")
    assert st["n_primaries"] == sum(sizes) and st["n_dropped"] == 0 and st["n_abandoned"] == 0
    assert abs(n_o - n_g) <= n_o - match and match >= MIN_MATCH * n_o, sorted(bad)[:10]
