"""Device-built model tables (csrc/grm_tables.hip, grm_model_init_device) against the host builders
(host/grm_host.cpp): hotcross (hotcross.cpp:60-79; the reference's GPU builder is
hotcross_table.cu:35-65), K2 (jnu_mixed.cpp:57-73; double-precision e^x K2(x) on the device, the
host uses std::cyl_bessel_k) and nint / dndlnu_max (harm_model.cpp:308-338).

The device sums every entry in the host's order with the host's grid and nodes; the remaining
differences are ocml vs glibc last bits (exp, log, pow) and K2's two evaluations.  The tables hold
logarithms, so an absolute difference is the relative difference of the tabulated quantity: K2
agrees to 1e-13 (measured ~4e-15: the device's trapezoid e^x K2(x) and std::cyl_bessel_k); nint and
dndlnu_max, sums of 200 interpolated emissivities over a weight table that itself comes from the
device K2, to 1e-11 (measured ~7e-13).  hotcross: the Klein-Nishina expression (hotcross.cpp:144-151)
cancels ~6 digits just above its w = 1e-3 switch, so a last-bit difference of its argument or of
log(1 + 2w) becomes ~1e-10 of sigma.  The device kernel therefore rounds every product and sum as the
host's build does (no FMA contraction: its 1 - mu v as one fma had put the argument an ulp off) and
takes that log correctly rounded (grm_crlog.h), as glibc's is but for arguments within ~0.005 ulp of
a rounding boundary, with the final log10 built as glibc builds it.  Measured: 2.14e-10 before (ocml
log, contraction; the log alone left that entry unchanged), 2.75e-12 with both, 0.848 of the entries
bit-identical (profiles/r05_tables_crlog.log); bar 3e-11, ten times that.  The table build takes
~31-37 ms of GPU time instead of 4.4 (a double-double exp per log below w = 0.1), once per model.  What is left is glibc's misrounded logs
(0.02 % of arguments, tests/test_crlog.py) in the cancelling range and ocml's exp in the
Maxwell-Juttner weights."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ulps(a, b):
    return np.abs(a - b) / np.spacing(np.maximum(np.abs(b), 1e-300))


def test_device_tables_match_host(dump32):
    import grmonty_amd as G
    host = G.Model.load(dump32, photon_n=1000).init(4)
    dev = G.Model.load(dump32, photon_n=1000).init(4, device=0)
    assert dev.table_ms > 0.0
    for which, name in ((0, "hotcross"), (1, "k2"), (4, "nint"), (5, "dndlnu_max")):
        h, d = host.table(which), dev.table(which)
        assert h.shape == d.shape and np.all(np.isfinite(d) == np.isfinite(h)), name
        f = np.isfinite(h)
        u = _ulps(d[f], h[f])
        print(f"{name}: {f.sum()} entries, max {u.max():.1f} ulp, bit-identical {np.mean(u == 0):.3f}, "
              f"max |diff| {np.max(np.abs(d[f] - h[f])):.3g}")
        if which == 0:
            k = int(np.argmax(np.abs(d - h)))
            print(f"  worst hotcross entry (w index, theta index) {divmod(k, 81)}: host {h.flat[k]!r} device {d.flat[k]!r}")
            assert np.max(np.abs(d[f] - h[f])) <= 3e-11 and np.mean(u == 0) > 0.8
        else:
            assert np.max(np.abs(d[f] - h[f])) <= (1e-13 if which == 1 else 1e-11), (name, np.max(np.abs(d[f] - h[f])))
    # the weight table is built on the host from the device K2: same to a few ulp
    h, d = host.table(3), dev.table(3)
    f = np.isfinite(h)
    assert np.array_equal(f, np.isfinite(d)) and np.max(np.abs(d[f] - h[f])) <= 1e-12
    print(f"device table build: {dev.table_ms:.2f} ms GPU time")
