"""Pin the CPU oracle before trusting it.

- tetrads / proba / monty_rand / integration: the REFERENCE's own sources are compiled here
  (oracle/Makefile -> oracle/_ref/libref_partial.so) and the oracle must agree bit for bit
  (same mt19937 seed, same libstdc++ distributions).
- GK61: the known answers of the reference's tests/integration_test.cpp:18-116.
- Philox4x32-10: Random123's published known-answer vectors.
The rest of the reference (harm_model/radiation/hotcross/jnu_mixed) needs spdlog + std::format,
absent from this image: those parts are pinned by independent mathematics in test_physics_pins.py.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O

DP = C.POINTER(C.c_double)
import os


class _LazyRef:
    """oracle/_ref/libref_partial.so, loaded on first use only (so a GPU-only test session, which
    collects this module but deselects its tests, never maps it)"""

    def __getattr__(self, name):
        return getattr(O.ref(), name)


HAVE_REF = os.path.exists(O.REF_PATH)
ref = _LazyRef() if HAVE_REF else None
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (reference tree absent)")


def _rng(seed):
    return O.lib().grmo_rng_new(0, seed, 0)


@needs_ref
def test_uniform_and_chi2_streams_bitexact():
    L = O.lib()
    g = _rng(123)
    ref.ref_rng_init(123)
    a = [L.grmo_rng_uniform(g) for _ in range(1000)]
    b = [ref.ref_uniform() for _ in range(1000)]
    assert a == b
    for dof in (3, 4, 5, 6):
        assert [L.grmo_rng_chi_sq(g, dof) for _ in range(200)] == [ref.ref_chi_sq(dof) for _ in range(200)]
    L.grmo_rng_free(g)


@needs_ref
@pytest.mark.parametrize("theta_e", [0.01, 0.3, 1.0, 7.5, 60.0, 400.0])
def test_electron_sampler_bitexact(theta_e):
    """proba::sample_electron_distr_p (proba.cpp:30-112) incl. chi^2 mixture rejection."""
    L = O.lib()
    g = _rng(99)
    ref.ref_rng_init(99)
    rng = np.random.default_rng(int(theta_e * 1000))
    for _ in range(400):
        k = rng.normal(size=4)
        k[0] = np.linalg.norm(k[1:])
        k *= 10 ** rng.uniform(-6, 1)
        k = np.ascontiguousarray(k)
        p1, p2 = np.zeros(4), np.zeros(4)
        L.grmo_sample_electron(g, k.ctypes.data_as(DP), p1.ctypes.data_as(DP), theta_e)
        ref.ref_sample_electron(k.ctypes.data_as(DP), p2.ctypes.data_as(DP), theta_e)
        assert np.array_equal(p1, p2)
    L.grmo_rng_free(g)


@needs_ref
def test_kn_thomson_dir_bitexact():
    L = O.lib()
    g = _rng(7)
    ref.ref_rng_init(7)
    for k0 in (1e-4, 1e-3, 0.05, 1.0, 30.0, 1e4):
        assert [L.grmo_sample_klein_nishina(g, k0) for _ in range(300)] == \
               [ref.ref_sample_klein_nishina(k0) for _ in range(300)]
    assert [L.grmo_sample_thomson(g) for _ in range(500)] == [ref.ref_sample_thomson() for _ in range(500)]
    for _ in range(300):
        a, b = np.zeros(3), np.zeros(3)
        L.grmo_sample_rand_dir(g, a.ctypes.data_as(DP))
        ref.ref_sample_rand_dir(b.ctypes.data_as(DP))
        assert np.array_equal(a, b)
    L.grmo_rng_free(g)


@needs_ref
def test_tetrad_bitexact(oracle64):
    """tetrads::make_tetrad (tetrads.cpp:68-124) on the synthetic dump's metric and fluid."""
    L = O.lib()
    rng = np.random.default_rng(0)
    h = oracle64.header
    for _ in range(300):
        x = np.array([0.0, rng.uniform(h.x_start[1], h.x_stop[1]), rng.uniform(0.02, 0.98), 0.0])
        f = np.zeros(1, dtype=O.FLUID)
        L.grmo_fluid_params(oracle64.h, x.ctypes.data_as(DP), f.ctypes.data_as(C.c_void_p))
        g = np.zeros(16)
        L.grmo_gcov(oracle64.h, x.ctypes.data_as(DP), g.ctypes.data_as(DP))
        u = np.ascontiguousarray(f["u_con"][0])
        tr = np.ascontiguousarray(f["b_con"][0] / (f["b"][0] / oracle64.units.b_unit))
        e1, l1, e2, l2 = (np.zeros(16) for _ in range(4))
        L.grmo_make_tetrad(u.ctypes.data_as(DP), tr.ctypes.data_as(DP), g.ctypes.data_as(DP),
                           e1.ctypes.data_as(DP), l1.ctypes.data_as(DP))
        ref.ref_make_tetrad(u.ctypes.data_as(DP), tr.ctypes.data_as(DP), g.ctypes.data_as(DP),
                            e2.ctypes.data_as(DP), l2.ctypes.data_as(DP))
        assert np.array_equal(e1, e2) and np.array_equal(l1, l2)
        # the tetrad is orthonormal in g
        G = g.reshape(4, 4)
        E = e1.reshape(4, 4)
        np.testing.assert_allclose(E @ G @ E.T, np.diag([-1, 1, 1, 1]), atol=1e-9)


GK_CASES = [  # (integrand code, a, b, expected) -- reference tests/integration_test.cpp:18-116
    (0, 0, 1, 1.0), (1, 0, 2, 6.0), (2, -1, 1, 4.0 / 3.0), (3, 0, np.pi, 2.0), (4, 0, 1, 0.29),
    (5, 0, 1, 2.0 / 3.0), (6, 1e-5, 1, -0.999874870746), (7, 0, np.pi, 0.0), (8, 0, 1, 0.0953512032278),
    (9, 0, 1, 0.5)]


@pytest.mark.parametrize("code,a,b,expected", GK_CASES)
def test_gk61_known_answers(code, a, b, expected):
    L = O.lib()
    v = L.grmo_gk61(code, 0.0, a, b, 1e-6, 1e-6, 1000)
    assert abs(v - expected) <= 1e-6
    if ref is not None:
        assert v == ref.ref_gk61(code, a, b, 1e-6, 1e-6, 1000)


def test_philox_known_answers():
    """Random123 philox4x32_10 KAT vectors."""
    L = O.lib()
    cases = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
             ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
             ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
              (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in cases:
        c = (C.c_uint32 * 4)(*ctr)
        k = (C.c_uint32 * 2)(*key)
        o = (C.c_uint32 * 4)()
        L.grmo_philox4x32(c, k, o)
        assert tuple(o) == want


def test_philox_uniform_and_chi2_distribution():
    """The device chi^2 construction (-2 ln prod u (+ z^2)) has the chi^2(dof) law."""
    from scipy import stats
    L = O.lib()
    g = L.grmo_rng_new(1, 123, 9)
    u = np.array([L.grmo_rng_uniform(g) for _ in range(20000)])
    assert u.min() > 0 and u.max() <= 1
    assert stats.kstest(u, "uniform").pvalue > 1e-3
    for dof in (3, 4, 5, 6):
        x = np.array([L.grmo_rng_chi_sq(g, dof) for _ in range(8000)])
        assert stats.kstest(x, "chi2", args=(dof,)).pvalue > 1e-3
    L.grmo_rng_free(g)


def test_oracle_reproduces_committed_reference_sampler_outputs():
    """tests/golden/ref_samplers.npz holds outputs of the REFERENCE's own proba.cpp (partial build,
    seed 123; tools/make_golden.py).  The oracle must reproduce them bit for bit -- this pin travels
    to machines without /root/reference."""
    import os
    L = O.lib()
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_samplers.npz"))
    g = L.grmo_rng_new(0, 123, 0)
    for i in range(len(d["k"])):
        k = np.ascontiguousarray(d["k"][i])
        p = np.zeros(4)
        L.grmo_sample_electron(g, k.ctypes.data_as(DP), p.ctypes.data_as(DP), float(d["theta_e"][i]))
        assert np.array_equal(p, d["p"][i]), i
    assert np.array_equal([L.grmo_sample_klein_nishina(g, float(v)) for v in d["k0"]], d["kn"])
    assert np.array_equal([L.grmo_sample_thomson(g) for _ in range(len(d["thomson"]))], d["thomson"])
    L.grmo_rng_free(g)
