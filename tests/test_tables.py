"""Init tables (harm_model.cpp:242-338, hotcross.cpp:60-79, jnu_mixed.cpp:57-73): the product's
multi-threaded C++ builders vs the oracle's serial restatement (bit-identical: same arithmetic,
same summation order), and the Bessel K2 table vs scipy (independent implementation)."""
import numpy as np
import pytest
from scipy.special import kv

NAMES = {0: "hotcross", 1: "k2", 2: "f", 3: "weight", 4: "nint", 5: "dndlnu_max", 6: "det"}


@pytest.mark.parametrize("which", list(NAMES))
def test_tables_bitexact_vs_oracle(model64, oracle64, which):
    a = model64.table(which)
    b = oracle64.table(which)
    assert a.shape == b.shape
    np.testing.assert_array_equal(a, b, err_msg=NAMES[which])


def test_k2_table_vs_scipy(model64):
    t = np.exp(np.arange(201) * (np.log(100 / 0.3) / 200) + np.log(0.3))
    np.testing.assert_allclose(model64.table(1), np.log(kv(2, 1.0 / t)), rtol=1e-13, atol=1e-13)


def test_hotcross_limits(model64):
    """log10(sigma/sigma_T): ~0 in the Thomson corner, Klein-Nishina suppression at high w."""
    hc = model64.table(0).reshape(221, 81)
    assert abs(hc[0, 0] - np.log10(0.665245873e-24)) < 1e-3      # w = 1e-12, theta = 1e-4: ~Thomson (quadrature)
    assert hc[220, 0] < hc[0, 0] - 3                                 # w = 1e6: KN suppressed
    assert np.all(np.isfinite(hc))
