"""BASELINE configs[3] -- 8 x MI355X, photon_n = 1e8 sharded -- exercised on one GPU: rank 0's
strided zone shard of the 8-rank photon_n = 1e8 job (grmonty_amd.zone_shards, as bench.py gives it
to rank 0 of 8), ~1.8e8 superphotons, with the job-wide counter path linked (eight engines' pass
counter blocks shared, grm_engine_link_peers: the kernels' bias_den reads all eight blocks, as
grm_engine_set_peers maps them over xGMI on the 8-GPU node).

Asserted (the reference keeps int32 device counters, super_photon.cu:41-46, 978-979 -- SURVEY Q7;
here every counter is u64):
  - nothing dropped or abandoned; every emitted photon tracked; tracked = primaries + children;
  - the transport-step counter past 2^32 (a 32-bit counter would have wrapped);
  - the u64 counters equal the spectrum's independent fp64 sums (nph = recorded, nscatt =
    scattered: integers below 2^53 add exactly in fp64);
  - the kernels' view of the job counters = the rank's own counters (the seven peers are idle);
  - the overflow path: launches counted (>= 1), overflowed children all tracked;
  - the shard's luminosity, scaled by its share of the job's photons, within 2 % of the
    photon_n = 1e6 oracle runs (tests/golden/oracle_synth192_pn1e6.json: 56.96 +- 0.05): the
    luminosity estimator is unbiased whatever the adaptive bias (the bias's job-size effect moves the
    counters, not L).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORLD = 8
PHOTON_N = 100_000_000


def test_rank0_shard_of_photon_n_1e8_job(dump_dir):
    import grmonty_amd as G
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)
    model = G.Model.load(path, photon_n=PHOTON_N).init(8, device=0)
    shards = G.zone_shards(model.zone_weights(), WORLD)
    z0, z1, st = shards[0]
    n_job = model.count(seed=123)
    n_shard = model.count(seed=123, z0=z0, z1=z1, stride=st)
    assert 1.5e8 < n_shard < 2.2e8 and 1.3e9 < n_job < 1.6e9, (n_shard, n_job)
    engines = [G.Engine(model, device=0) for _ in range(WORLD)]
    try:
        for e in engines:
            e.stash_reserve(1)
        G.link_peers(engines)
        e = engines[0]
        e.emit_setup(model)
        e.begin_pass(0)
        e.set_option(G.OPT_SEED, 123)
        e.set_option(G.OPT_ID_BASE, 0)
        p, n = e.emit(seed=123, z0=z0, z1=z1, stride=st)
        assert n == n_shard
        e.track_device(p, n)
        s = e.stats()
        spec, n_rec, n_scatt, max_tau = e.finish()
        view = e.job_counters()
    finally:
        for x in engines:
            x.close()
    print(f"rank 0 of {WORLD}, photon_n {PHOTON_N:g}: {n} primaries, {s['n_tracked']} tracked, {n_rec} recorded, "
          f"{n_scatt} scattered, {s['n_steps']} steps, {s['n_launches']} launches, overflow {s['n_overflow']}, "
          f"lone {s['n_lone']}, early {s['n_early']}, longest life {s['max_photon_steps']}, "
          f"{s['last_kernel_ms']:.0f} ms")
    assert s["n_dropped"] == 0 and s["n_abandoned"] == 0
    assert s["n_primaries"] == n
    assert s["n_tracked"] == s["n_primaries"] + s["n_children"]
    assert s["n_steps"] > 2 ** 32
    assert s["n_launches"] >= 1
    assert float(spec["nph"].sum()) == float(n_rec)
    assert float(spec["nscatt"].sum()) == float(n_scatt)
    assert view["n_recorded"] == n_rec and view["n_scatt"] == n_scatt and view["max_tau_scatt"] == max_tau
    lum = model.write_spectrum(spec, None)["luminosity"]
    o = json.load(open(os.path.join(HERE, "golden", "oracle_synth192_pn1e6.json")))["runs"]
    l_ref = float(np.mean([r["luminosity"] for r in o]))
    scaled = lum * n_job / n
    print(f"luminosity: shard {lum:.4f}, x job/shard photons {scaled:.4f}, oracle photon_n=1e6 {l_ref:.4f} "
          f"({scaled / l_ref - 1:+.2%})")
    assert abs(scaled / l_ref - 1) < 0.02
