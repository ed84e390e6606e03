"""Emission (harm_model.cpp:673-811 get_zone / sample_zone_photon, :1337-1389 init_zone) with the
product's stream definition: per-zone count draw, then one Philox stream per photon.

The oracle restates the reference's zone walk and sampler (oracle/grmonty_oracle.cpp
grmo_emit_philox) and is driven by the same streams, so the product's C++ host emitter
(grm_model_emit) must agree with it bit for bit: same tables, same glibc arithmetic.  The zone table
that the GPU emitter consumes (grm_model_zone_table) is checked against the oracle's init_zone.
No GPU needed."""
import numpy as np

import grmonty_amd as G

FIELDS = ["x", "k", "w", "e", "l", "n_e_0", "theta_e_0", "b_0", "e_0", "n_scatt"]


def test_host_emission_bitexact_vs_oracle(model64, oracle64):
    for seed in (99, 123):
        ph = model64.emit(seed=seed)
        po = oracle64.emit_philox(seed=seed)
        assert len(ph) == len(po) > 10000
        for f in FIELDS:
            np.testing.assert_array_equal(ph[f], po[f], err_msg=f)


def test_emission_depends_only_on_seed(model64):
    a = model64.emit(seed=5, threads=1)
    b = model64.emit(seed=5, threads=7)
    assert a.tobytes() == b.tobytes()
    c = model64.emit(seed=6)
    assert len(c) != len(a) or a.tobytes() != c.tobytes()


def test_zone_shards_concatenate_to_the_whole_walk(model64):
    full = model64.emit(seed=11)
    shards = G.shard_zones(model64.zone_weights(), 3)
    parts = [model64.emit(seed=11, z0=a, z1=b) for a, b in shards]
    assert sum(len(p) for p in parts) == len(full)
    assert np.concatenate(parts).tobytes() == full.tobytes()
    for (a, b), p in zip(shards, parts):
        assert model64.count(seed=11, z0=a, z1=b) == len(p)


def test_zone_table_vs_oracle_init_zone(model64, oracle64):
    zt = model64.zone_table()
    h = model64.header
    n1, n2 = h.n[0], h.n[1]
    assert zt.shape == (n1 * n2,) and G.EMIT_ZONE.itemsize == 272 == G.lib().grm_sizeof(6)
    ref = np.array([oracle64.init_zone(i, j) for i in range(n1) for j in range(n2)])
    np.testing.assert_array_equal(zt["nz"], ref[:, 0])
    np.testing.assert_array_equal(zt["dn_max"], ref[:, 1])
    # zone centres (get_coord, harm_model.cpp:1639-1644) and tetrads orthonormal in the zone metric
    i, j = 10, 17
    z = zt[i * n2 + j]
    assert z["x"][1] == h.x_start[1] + (i + 0.5) * h.dx[1] and z["x"][2] == h.x_start[2] + (j + 0.5) * h.dx[2]
    # tetrad (make_tetrad, tetrads.cpp:68-124): orthonormal in the zone metric, e_cov = eta e_con g
    import ctypes as C
    import oracle_py as O
    g = np.zeros(16)
    x = np.ascontiguousarray(z["x"])
    O.lib().grmo_gcov(oracle64.h, x.ctypes.data_as(O.DP), g.ctypes.data_as(O.DP))
    g = g.reshape(4, 4)
    e_con = z["e_con"]
    eta = np.diag([-1.0, 1.0, 1.0, 1.0])
    np.testing.assert_allclose(e_con @ g @ e_con.T, eta, atol=1e-10)
    e_cov = eta @ e_con @ g
    np.testing.assert_allclose(z["e_cov_t"], e_cov[:, 0], rtol=1e-12, atol=1e-14 * np.abs(e_cov).max())
    np.testing.assert_allclose(z["e_cov_z"], e_cov[:, 3], rtol=1e-12, atol=1e-14 * np.abs(e_cov).max())
    assert C.sizeof(C.c_double) == 8


def test_zone_table_subrange(model64):
    full = model64.zone_table()
    part = model64.zone_table(100, 300)
    assert part.tobytes() == full[100:300].tobytes()
