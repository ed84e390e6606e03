"""The oracle's concurrency emulator (grmo_track_concurrent, oracle/grmonty_oracle.cpp): the
reference's track_super_photon (harm_model.cpp:894-1069) cut at its loop boundary and scheduled the
way a concurrent engine schedules it.  Its W = 1 setting must BE the serial reference: one slot,
children tracked depth-first in their parent's slot (the recursion at :1023), counters visible to
bias_func (:1391-1404) from the next round on -- operation for operation the serial loop, so the end
records, counters and spectrum are bit-identical to grmo_track_batch with the live bias.  With many
slots it is a valid run of the same estimator (every photon tracked, luminosity within the seed
spread).  CPU only."""
import numpy as np

import oracle_py as O


def _reset(m, mt0):
    m.reset()
    m.L.grmo_model_set_max_tau_scatt(m.h, mt0)


def test_one_slot_depth_first_is_the_serial_reference(oracle64):
    m = oracle64
    mt0 = m.scalars()["max_tau_scatt"]
    ph = m.emit_philox(seed=321)
    ph = ph[np.random.default_rng(1).permutation(len(ph))[:3000]]  # all zones, not only the innermost
    _reset(m, mt0)
    tr_s = m.track(ph, rng_mode=1, seed=321, frozen=False, trace_cap=200_000)
    c_s, s_s, mt_s = m.counters(), m.spectrum(), m.scalars()["max_tau_scatt"]
    _reset(m, mt0)
    rounds, tr_c, _ = m.track_concurrent(ph, seed=321, trace_cap=200_000)
    c_c, s_c, mt_c = m.counters(), m.spectrum(), m.scalars()["max_tau_scatt"]
    _reset(m, mt0)
    assert c_s == c_c and c_s["created"] == len(ph) and c_s["scattered"] > 0
    assert mt_s == mt_c > mt0
    assert len(tr_s) == len(tr_c) > len(ph)
    assert tr_s.tobytes() == tr_c.tobytes()
    assert s_s.tobytes() == s_c.tobytes()
    assert rounds >= c_s["steps"]


def test_many_slots_track_every_photon(oracle64):
    """device-like scheduling (4096 slots, wave stacks of 64, deferred children, counter snapshots
    every 64 rounds, interleaved claims, warm-up admission): every photon and child ends exactly
    once, and the records agree with the counters"""
    m = oracle64
    mt0 = m.scalars()["max_tau_scatt"]
    ph = m.emit_philox(seed=322)
    ph = ph[np.random.default_rng(2).permutation(len(ph))[:3000]]
    cfg = dict(O.OracleModel.EMU_DEVICE, slots=4096, warm_n=1024)
    _reset(m, mt0)
    _, tr, tl = m.track_concurrent(ph, seed=322, trace_cap=400_000, timeline_cap=4096, **dict(cfg, timeline=8))
    c = m.counters()
    _reset(m, mt0)
    assert c["created"] == len(ph)
    ids = tr["id"]
    assert len(np.unique(ids)) == len(ids)                     # every photon ends once
    prim = tr[tr["parent_id"] == np.uint64(2 ** 64 - 1)]
    assert len(prim) == len(ph) and set(prim["id"].tolist()) == set(range(len(ph)))
    kids = tr[tr["parent_id"] != np.uint64(2 ** 64 - 1)]
    assert set(kids["parent_id"].tolist()) <= set(ids.tolist())  # every child's parent ended too
    assert (tr["end_reason"] == 0).sum() == c["recorded"]
    # the timeline: claims and records only grow; nothing in flight at the end
    assert len(tl) > 3 and np.all(np.diff(tl[:, 1]) >= 0) and np.all(np.diff(tl[:, 2]) >= 0)
