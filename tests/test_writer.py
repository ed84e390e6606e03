"""Spectrum writer fidelity (report_spectrum, harm_model.cpp:416-471).

1. Column format: the reference writes std::format("{:10.5g} ", v); the product writes
   "%10.5g ".  For finite doubles the two are byte-identical -- checked here against fmt 12 (the
   library std::format was standardised from; libstdc++ 11 has no <format>) on edge forms (zeros of
   both signs, denormals, the largest double, 5-significant-digit rounding boundaries, exponent
   switch points) and 2,000 random magnitudes.  Non-finite values: the C++ standard right-aligns
   arithmetic types ([format.string.std]), so std::format writes "       nan" like printf; fmt 12
   left-aligns them (a library quirk, not the reference's std::format).  The spectrum cannot hold
   them anyway (record_super_photon drops NaN photons, every column divides by dn_dle + eps).
2. File bytes: the product's grm_write_spectrum and the oracle's report_spectrum restatement on the
   same spectrum (the oracle's seed-123 run at the headline scale, tests/golden) are identical, and
   so are luminosity and max tau_scatt.
3. The statistics sidecar (nph, dn_dle, de_dle per cell) round-trips the spectrum exactly.
"""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "oracle_synth192_pn1e5.npz")


def _fmt_include():
    try:
        import torch
        d = os.path.join(os.path.dirname(torch.__file__), "include")
        return d if os.path.exists(os.path.join(d, "fmt", "format.h")) else None
    except Exception:
        return None


def edge_values():
    v = [0.0, -0.0, 1.0, -1.0, 1e-300, 5e-324, 2.2250738585072014e-308, 1e300, 1.7976931348623157e308,
         123456.0, 99999.5, 99999.4, 9.99995, 9.99994999, 0.0001, 0.00001, 0.000012345678, 1e5, 1e-5, 1e-4,
         99999.95, -2.5e-7, 1.5, 3.14159265, 0.5, 12345.5, 1234.55, 0.000099999, -123456789.0, 1e16, 1e-16,
         0.00009999951, 999995.0, 2.5, -0.000123456]
    rng = np.random.default_rng(0)
    v += list(10.0 ** rng.uniform(-320, 308, 2000) * rng.choice([-1, 1], 2000))
    return v


def test_format_matches_std_format_semantics(tmp_path):
    inc = _fmt_include()
    if inc is None or shutil.which("g++") is None:
        pytest.skip("fmt headers / g++ not available")
    exe = str(tmp_path / "fmtchk")
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{inc}", os.path.join(HERE, "native", "fmt_vs_printf.cpp"), "-o",
                    exe], check=True)
    vals = edge_values() + [float("nan"), -float("nan"), float("inf"), -float("inf")]
    inp = "\n".join("%016x" % struct.unpack("<Q", struct.pack("<d", x))[0] for x in vals) + "\n"
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    assert len(out) == len(vals)
    for x, line in zip(vals, out):
        a, b = line.split("|")
        if np.isfinite(x):
            assert a == b, (x, a, b)
        else:
            # std::format right-aligns arithmetic types: "{:10.5g}" of nan is "       nan" == printf
            assert b == ("%10s " % (("-" if np.signbit(x) else "") + ("nan" if np.isnan(x) else "inf")))


@pytest.fixture(scope="module")
def golden_spectrum():
    if not os.path.exists(GOLD):
        pytest.skip("headline-scale golden not generated (tools/make_golden_192.py)")
    g = np.load(GOLD)
    import oracle_py as O
    spec = np.ascontiguousarray(g["spectrum123"].reshape(-1)).view(O.SPECTRUM_CELL)
    return spec


def test_writer_bytes_equal_oracle(tmp_path, dump32, golden_spectrum):
    import grmonty_amd as G
    import oracle_py as O
    # the writer depends on the header's x2 range and h_slope only: the 192x192 and the 32x48
    # synthetic dumps share them, so the small dump keeps the model set-up cheap
    m = G.Model.load(dump32, photon_n=100).init(2)
    o = O.OracleModel(dump32, photon_n=100)
    o.set_spectrum(golden_spectrum)
    po, pp = str(tmp_path / "oracle.spec"), str(tmp_path / "product.spec")
    ro = o.report(po)
    rp = m.write_spectrum(golden_spectrum.view(G.SPECTRUM_CELL), pp)
    bo, bp = open(po, "rb").read(), open(pp, "rb").read()
    assert bo == bp
    assert ro["luminosity"] == rp["luminosity"] and ro["max_tau_scatt"] == rp["max_tau_scatt"]
    rows = bp.decode().split("\n")
    assert rows[-1] == "" and len(rows) == 201
    for r in rows[:-1]:
        assert r.endswith(" ")            # every field is followed by one space, then the newline
        assert len(r.split()) == 37       # log10 E + 6 theta bins x 6 columns
    assert rp["luminosity"] > 0


def test_stats_sidecar_roundtrip(tmp_path, dump32, golden_spectrum):
    import grmonty_amd as G
    m = G.Model.load(dump32, photon_n=100).init(2)
    p = str(tmp_path / "spec.stats")
    spec = golden_spectrum.view(G.SPECTRUM_CELL).reshape(6, 200)
    m.write_spectrum_stats(spec, p)
    a = np.loadtxt(p)
    assert a.shape == (200, 1 + 6 * 3)
    for j in range(6):
        np.testing.assert_array_equal(a[:, 1 + 3 * j], spec["nph"][j])
        np.testing.assert_array_equal(a[:, 2 + 3 * j], spec["dn_dle"][j])
        np.testing.assert_array_equal(a[:, 3 + 3 * j], spec["de_dle"][j])
    np.testing.assert_allclose(a[:, 0], (np.arange(200) * 0.25 + np.log(1e-12)) / np.log(10), rtol=1e-15)
